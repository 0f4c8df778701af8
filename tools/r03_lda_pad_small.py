"""The reference's sizes (N = 4096, 8192): k_matvec_f64 through the
kernel-level cgx_matvec with the row pitch lda = N + pad, timed per launch
with back-to-back launches (GPU only).  Does a non-power-of-two pitch help
when 2048 concurrent rows sit at the same column offset?"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import conjugate_gradient_amd as cg  # noqa: E402

PADS = [0, 64, 128, 256]
lib = cg.lib()
for N in (8192, 4096):
    A = cg.DeviceArray(N * (N + max(PADS)))
    v = cg.DeviceArray(N + max(PADS))
    out = cg.DeviceArray(N)
    for p in PADS:
        cg.matVec(A, v, out, N, N, lda=N + p)
    lib.cgx_dev_synchronize()
    for rnd in range(3):
        for p in PADS:
            reps = 400
            t0 = time.perf_counter()
            for _ in range(reps):
                cg.matVec(A, v, out, N, N, lda=N + p)
            lib.cgx_dev_synchronize()
            us = (time.perf_counter() - t0) / reps * 1e6
            print(json.dumps({"n": N, "round": rnd, "pad": p, "us": round(us, 2),
                              "gbps": round(8 * N * N / (us * 1e-6) / 1e9, 1)}), flush=True)
    A.free()
