import cProfile, pstats, sys, os, io
sys.argv = ["bench_workloads.py", "--workload", "config3", "--steps", "30"]
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "scripts")]
import bench_workloads as bw
pr = cProfile.Profile()
orig = bw.timed
def timed(step, steps, warmup):
    step(); step(); step()
    import torch; torch.cuda.synchronize()
    pr.enable()
    for _ in range(steps): step()
    torch.cuda.synchronize()
    pr.disable()
    return orig(step, 5, 1)
bw.timed = timed
bw.main()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
print(s.getvalue())
