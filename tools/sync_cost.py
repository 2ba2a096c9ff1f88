"""Fixed costs around a short timed region on the GPU box: how long an idle torch.cuda.synchronize()
takes, how long the host needs to notice a finished event, and the start latency of a graph replay
vs a direct launch, measured with the bench's own step kernel (65 536 envs, W=10)."""
import ctypes as C
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import gym_ballenv_amd as gb  # noqa: E402
from gym_ballenv_amd import _abi  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N, W, K = 65536, 10, 20
env = gb.BatchedBallEnv(N, W, gb.EnvConfig(), device=dev, seed=0xBA11)
acts = env.sample_actions(K, seed=1)
env.reset()
lib, ctx, st, out = _abi.lib(), env._ctx, C.byref(env._st), C.byref(env._out)
stream = torch.cuda.current_stream(dev)
sp = C.c_void_p(stream.cuda_stream)


def med(f, n=200):
    ts = []
    for _ in range(n):
        ts.append(f())
    return statistics.median(ts) * 1e6


def idle_sync():
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0


def idle_stream_sync():
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    stream.synchronize()
    return time.perf_counter() - t0


def idle_query():
    torch.cuda.synchronize(dev)
    e = torch.cuda.Event()
    e.record(stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e.query()
    return time.perf_counter() - t0


print("idle torch.cuda.synchronize  %.2f us" % med(idle_sync))
print("idle stream.synchronize      %.2f us" % med(idle_stream_sync))
print("event.query (done)           %.2f us" % med(idle_query))

g = torch.cuda.CUDAGraph()
cap = torch.cuda.Stream(dev)
with torch.cuda.graph(g, stream=cap):
    cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for t in range(K):
        lib.be_step(ctx, st, C.c_void_p(acts[t].data_ptr()), None, None, out, cs)
g.replay()
torch.cuda.synchronize(dev)


def region(kind, end):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    t0 = time.perf_counter()
    if kind == "graph":
        g.replay()
    elif kind == "loop":
        lib.be_step_n(ctx, st, C.c_void_p(acts.data_ptr()), K, out, sp)
    ev1.record(stream)
    if end == "spin":
        while not ev1.query():
            pass
        torch.cuda.synchronize(dev)
    elif end == "stream":
        stream.synchronize()
        torch.cuda.synchronize(dev)
    else:
        torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    return el, ev0.elapsed_time(ev1) * 1e3


hip = C.CDLL("libamdhip64.so")
hip.hipGraphLaunch.argtypes = [C.c_void_p, C.c_void_p]
gexec = C.c_void_p(g.raw_cuda_graph_exec())


def host_call(kind):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if kind == "graph":
        g.replay()
    else:
        assert hip.hipGraphLaunch(gexec, sp) == 0
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    return t1 - t0


print("host time of g.replay()          %.2f us" % med(lambda: host_call("graph"), 50))
print("host time of hipGraphLaunch()    %.2f us" % med(lambda: host_call("raw"), 50))


def region_raw():
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    ev0.record(stream)
    t0 = time.perf_counter()
    assert hip.hipGraphLaunch(gexec, sp) == 0
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0, ev0.elapsed_time(ev1) * 1e3


r = [region_raw() for _ in range(30)]
print("raw   end=sync   wall %.1f us  events %.1f us" % (statistics.median(x for x, _ in r) * 1e6,
                                                         statistics.median(y for _, y in r)))
def capture(t0, t1):
    gg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gg, stream=cap):
        cs = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for t in range(t0, t1):
            lib.be_step(ctx, st, C.c_void_p(acts[t].data_ptr()), None, None, out, cs)
    gg.replay()
    torch.cuda.synchronize(dev)
    return gg


for head in (1, 2, 4):
    parts = [capture(0, head), capture(head, K)]

    def region_split():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        t0 = time.perf_counter()
        for gg in parts:
            gg.replay()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0, ev0.elapsed_time(ev1) * 1e3

    r = [region_split() for _ in range(30)]
    print("split %d+%d  wall %.1f us  events %.1f us" % (head, K - head, statistics.median(x for x, _ in r) * 1e6,
                                                       statistics.median(y for _, y in r)))
for kind in ("graph", "loop"):
    for end in ("spin", "stream", "sync"):
        r = [region(kind, end) for _ in range(30)]
        print("%-5s end=%-6s wall %.1f us  events %.1f us  (K=%d, median of 30)" % (
            kind, end, statistics.median(x for x, _ in r) * 1e6, statistics.median(y for _, y in r), K))
env.close()
