# symmetric storage: contiguous vs interleaved unit walk on the same allocation of A, over fresh allocations
import json, os, sys, time
sys.path.insert(0, '/root/repo')
import conjugate_gradient_amd as cg
n = 65536
keep = []
for k in range(6):
    res = {}
    with cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_SYMMETRIC) as s:
        s.generate_spd(42); s.begin(); s.iterate(3, eps=-1.0); s.synchronize()
        for rep in range(2):
            for walk in (0, 1):
                os.environ["CGX_SYM_PLAN"] = f"walk={walk}"
                s.iterate(2, eps=-1.0); s.synchronize()
                t0 = time.perf_counter(); s.iterate(20, eps=-1.0); s.synchronize(); t1 = time.perf_counter()
                res.setdefault(f"walk{walk}", []).append(round(20 / (t1 - t0), 1))
    print(json.dumps({"alloc": k, **res}), flush=True)
    keep.append(cg.DeviceArray(((k + 1) * 37) << 20))
