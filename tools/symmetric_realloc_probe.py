# symmetric storage: the iteration rate after each fresh allocation of A within one process
# (round 5's probe behind profiles/r05_symmetric_realloc.jsonl)
import json, sys, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import conjugate_gradient_amd as cg
n = 65536
pad = []
for k in range(8):
    with cg.Solver(n, flags=cg.CGX_F64 | cg.CGX_SYMMETRIC) as s:
        s.generate_spd(42); s.begin(); s.iterate(3, eps=-1.0); s.synchronize()
        t0 = time.perf_counter(); s.iterate(20, eps=-1.0); s.synchronize(); t1 = time.perf_counter()
    print(json.dumps({"alloc": k, "it_s": round(20 / (t1 - t0), 1)}), flush=True)
    if k % 2 == 0:  # shift the next allocation: hold a small buffer
        p = cg.DeviceArray(((k + 1) * 37) << 20)  # (k+1)*37 Mi doubles
        pad.append(p)
