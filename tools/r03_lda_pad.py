"""Dense matVec (k_matvec_f64, the library's default plan, through the
kernel-level cgx_matvec) over 65536 rows x 65536 columns with the row pitch
lda = 65536 + pad: does a pitch that is not a power of two (rows starting at
different offsets modulo the HBM channel interleave) read faster?  GPU only;
one buffer of 65536 x (65536 + max pad) doubles, pads interleaved."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

N = 65536
PADS = [0, 64, 128, 256, 512]
A = cg.DeviceArray(N * (N + max(PADS)))
v = cg.DeviceArray(N)
out = cg.DeviceArray(N)
lib = cg.lib()
for p in PADS:  # warm-up each pitch once
    cg.matVec(A, v, out, N, N, lda=N + p)
lib.cgx_dev_synchronize()
for rnd in range(3):
    for p in PADS:
        t0 = time.perf_counter()
        for _ in range(10):
            cg.matVec(A, v, out, N, N, lda=N + p)
        lib.cgx_dev_synchronize()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        print(json.dumps({"round": rnd, "pad": p, "ms": round(ms, 4),
                          "gbps": round((8 * N * N + 16 * N) / (ms * 1e-3) / 1e9, 1)}), flush=True)
