# Host-cost A/B of two libballenv.so builds: tools/hostab/libballenv.so (the baseline: copy a build there
# first; *.so stays out of git) against the in-tree one -- be_step from C (tools/step_host), then the
# bench legs with the eager_step leg (tools/ab.sh).  profiles/r06_launch_host_ab.txt.
set -u
mkdir -p gpurun_out
for r in 1 2 3 4 5; do
  echo "old r$r: $(LD_LIBRARY_PATH=tools/hostab timeout -k 10 60 ./tools/step_host | head -1)" || exit 1
  echo "new r$r: $(timeout -k 10 60 ./tools/step_host | head -1)" || exit 1
done
ARMS="old new" LIB_old=tools/hostab/libballenv.so EXTRA="--eager-steps 1000" REPS=3 TAG=hostab bash tools/ab.sh || exit 1
for f in gpurun_out/hostab/*.log; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); e=d['eager_step']
print('$f', 'eager host us/call %.3f  us/iter %.3f' % (e['host_us_per_step_call'], e['host_us_per_iteration']))"; done
