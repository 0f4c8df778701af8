"""One rank of a multi-rank RCCL job on a single GPU (tests/test_gpu_multirank.py).

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected");
the parent gives every rank its own NCCL_HOSTID, so RCCL sees P hosts and
carries the exchange over its socket transport on the loopback interface.
The data path is then host-staged instead of xGMI, but everything libcgx does
in rank mode runs at world size P: the in-place ncclAllGather into each
rank's row-block slot, the scalar allreduces, the overlapped exchange on the
comm stream, the p2p pattern, the rank-ordered combine, the Poisson halo
ncclSend/Recv, and the final x allgather.

  python tests/_rank_worker.py MODE N P RANK UIDFILE OUTPREFIX
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import conjugate_gradient_amd as cg  # noqa: E402
import oracle  # noqa: E402
from _cases import case  # noqa: E402


def main():
    mode, n, P, rank, uidfile, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        sys.argv[5], sys.argv[6]
    if rank == 0:
        uid = cg.get_unique_id()
        with open(uidfile + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(uidfile + ".tmp", uidfile)
    else:
        t0 = time.time()
        while not os.path.exists(uidfile):
            if time.time() - t0 > 60:
                raise SystemExit("no unique id from rank 0")
            time.sleep(0.05)
        with open(uidfile, "rb") as f:
            uid = f.read()
    res = {"rank": rank}
    if mode in ("peer_dies", "peer_absent", "poisson_peer_dies"):
        return fail_fast(mode, n, P, rank, uid, out)
    # one GPU per rank where the box has them (tests/test_gpu_multidevice.py), else all on device 0
    dev = rank if os.environ.get("CGX_TEST_RANK_DEVICE") == "rank" else 0
    if mode.startswith("poisson"):
        m = n
        with cg.Solver(None, poisson_m=m, rank=rank, nranks=P, unique_id=uid, device=dev) as s:
            res["comm"] = s.comm_info()
            s.fill(1.0, 0.0)
            eps = 1e-8 if mode == "poisson_eps" else -1.0
            x, st = s.solve(None, eps=eps, max_iter=-1 if eps > 0 else 120)
            res.update(iterations=st.iterations, converged=st.converged)
    else:
        flags = {"f32ref": cg.CGX_F32_REF, "p2p": cg.CGX_COMM_P2P, "nooverlap": cg.CGX_NO_OVERLAP,
                 "deterministic": cg.CGX_DETERMINISTIC, "headline_det": cg.CGX_DETERMINISTIC,
                 "det_overlap": cg.CGX_DETERMINISTIC,
                 "p2p_f32ref": cg.CGX_F32_REF | cg.CGX_COMM_P2P}.get(mode, cg.CGX_F64)
        if not flags & cg.CGX_F32_REF:
            flags |= cg.CGX_F64
        f32 = bool(flags & cg.CGX_F32_REF)
        if mode.startswith("headline"):  # configs[2]: the bench's N=65536 system, generated on the device
            A = b = x0 = None
        elif mode == "sized":  # any n: generateSPDmatrix(n) from the oracle's MATLAB-compatible generator
            A, b = oracle.spd_matlab(n, np.float64)
            x0 = np.zeros(n)
        else:
            A, b, x0 = case(f"spd{n}", np.float32 if f32 else np.float64)
        if mode in ("overlap_on", "det_overlap"):  # the overlapped form whatever the measurement says
            os.environ["CGX_OVERLAP"] = "1"
        with cg.Solver(n, rank=rank, nranks=P, unique_id=uid, device=dev, flags=flags) as s:
            res["comm"] = s.comm_info()
            res["overlap"] = bool(s.info.flags & cg.CGX_OVERLAP_ACTIVE)
            res["overlap_info"] = s.overlap_info()
            res["nrows"] = s.info.nrows
            if A is None:
                s.generate_spd(42)
            else:
                s.set_system(A, b, x0)
            x, st = s.solve(None, eps=1e-6 if f32 else 1e-10)
            rn, bn = s.residual_norm()
            res.update(iterations=st.iterations, converged=st.converged, relres=rn / bn)
            if mode == "collective":  # a fixed-count run from a nonzero x0 (initial exchange + matVec)
                s.set_x(np.full(n, 0.25))
                _, st2 = s.solve(None, eps=-1.0, max_iter=5)
                res["fixed_iterations"] = st2.iterations
                res["fixed_relres"] = float(np.divide(*s.residual_norm()))
    np.save(out + f"_x{rank}.npy", x)
    with open(out + f"_r{rank}.json", "w") as f:
        json.dump(res, f)


def fail_fast(mode, n, P, rank, uid, out):
    """Rank mode must fail fast, not hang, when a peer is gone (the reference
    stops the job with MPI_Abort, parallel_cg.c:79,89,94,143).
      peer_dies:   the last rank exits right after cgx_create_rank; the others
                   set up and solve, and must get CGX_ERR_RCCL within the deadline.
      peer_absent: the last rank never creates its context; the others must get
                   CGX_ERR_RCCL from cgx_create_rank within the deadline.
      poisson_peer_dies: peer_dies on an m = n Poisson grid, x deferred over
                   iterations (the default): after the failed iterate, x is
                   refused (CGX_ERR_STATE) instead of handed out incomplete."""
    poisson = mode == "poisson_peer_dies"
    if rank == P - 1:
        if mode == "peer_dies":
            cg.Solver(n, rank=rank, nranks=P, unique_id=uid, device=0)
        if poisson:  # joins the solve's start (its collectives), then dies before the iterations
            s = cg.Solver(None, poisson_m=n, rank=rank, nranks=P, unique_id=uid, device=0)
            s.fill(1.0, 0.0)
            s.begin()
            s.synchronize()
        os._exit(0)  # no destroy, no finalisation: as if the process died
    if poisson:
        return fail_fast_poisson(n, P, rank, uid, out)
    A, b, x0 = case(f"spd{n}", np.float64)
    t0 = time.time()
    res = {"rank": rank, "error": None}

    def say(msg):
        print(f"[rank {rank} +{time.time() - t0:.1f}s] {msg}", flush=True)

    s = None
    try:
        say("cgx_create_rank")
        s = cg.Solver(n, rank=rank, nranks=P, unique_id=uid, device=0)
        res["created_s"] = time.time() - t0
        say("set_system + solve")
        s.set_system(A, b, x0)
        res["failed_in"] = "cgx_solve_begin"
        s.begin()
        res["failed_in"] = "cgx_iterate"
        s.iterate(n, eps=1e-10)
        res["failed_in"] = None
    except cg.CgxError as e:
        res.update(error=str(e), code=e.code)
        say(f"error: {e}")
        if s is not None:  # after a failed iterate x may hold part of an iteration: refused
            try:
                s.get_x()
                res["get_x"] = "ok"
            except cg.CgxError as e2:
                res.update(get_x=str(e2), get_x_code=e2.code)
    res["elapsed_s"] = time.time() - t0
    with open(out + f"_r{rank}.json", "w") as f:
        json.dump(res, f)
    if s is not None:
        say("cgx_destroy")
        try:
            s.close()
        except cg.CgxError as e:
            say(f"destroy: {e}")
    say("exit")
    os._exit(0)  # as bench.py does after an error: no teardown that could wait on the dead peer


def fail_fast_poisson(m, P, rank, uid, out):
    t0 = time.time()
    res = {"rank": rank, "error": None}
    s = cg.Solver(None, poisson_m=m, rank=rank, nranks=P, unique_id=uid, device=0)
    res["created_s"] = time.time() - t0
    res["xdefer"] = bool(s.info.flags & cg.CGX_XDEFER_ACTIVE)
    s.fill(1.0, 0.0)
    try:
        s.begin()
        s.iterate(200, eps=1e-12)
    except cg.CgxError as e:
        res.update(error=str(e), code=e.code)
    try:
        s.get_x()
        res["get_x"] = "ok"
    except cg.CgxError as e:
        res.update(get_x=str(e), get_x_code=e.code)
    res["elapsed_s"] = time.time() - t0
    with open(out + f"_r{rank}.json", "w") as f:
        json.dump(res, f)
    os._exit(0)


if __name__ == "__main__":
    main()
