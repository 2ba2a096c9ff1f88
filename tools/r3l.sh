set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for B in noacos noexp nohypot noall; do B=$B bash tools/board_ab.sh 2>&1 | tail -4 || exit 1; done
