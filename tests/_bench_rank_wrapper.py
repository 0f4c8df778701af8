"""bench.py as one rank of a torchrun job on a one-GPU box (tests/test_gpu_multirank.py).

Every rank gets its own NCCL_HOSTID (RCCL then uses its socket transport
instead of refusing two ranks on one device) and drives GPU 0; the rest is
bench.py unchanged: gloo control plane, cgx_create_rank, barrier-bracketed
timed region, max over ranks, one JSON line from rank 0.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

os.environ["NCCL_HOSTID"] = "cgx-bench-host-" + os.environ.get("RANK", "0")
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
os.environ["LOCAL_RANK"] = "0"  # one GPU: every rank drives device 0

import bench  # noqa: E402

if __name__ == "__main__":
    sys.exit(bench.run())
