"""Interleaved A/B of environment variants on one bench workload (GPU box,
repo root): every round runs each variant once, in a separate bench.py
process, so a slow box or process-to-process drift hits every variant alike.

  python tools/ab_variants.py --rounds 2 --args "--workload poisson --steps 300" \
      --variant default= --variant grid1024=CGX_POISSON_PLAN=blocks=1024 > out.jsonl

A variant is NAME=VAR=VALUE[,VAR=VALUE...] (NAME= alone: the defaults).
Each line: the variant, the round, it/s, the roofline figure, relres."""
import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_variant(text):
    name, _, rest = text.partition("=")
    env = {}
    for item in filter(None, rest.split(",")):
        k, _, v = item.partition("=")
        env[k] = v
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--args", default="", help="bench.py arguments (--no-cpu is added)")
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    variants = [parse_variant(v) for v in a.variant]
    for r in range(a.rounds):
        for name, env in variants:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu"] + shlex.split(a.args)
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, env=dict(os.environ, **env))
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                sys.exit(p.returncode)
            d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
            print(json.dumps({"variant": name, "env": env, "round": r, "value": round(d["value"], 2),
                              "ms_per_step": round(d["ms_per_step"], 4),
                              "roofline_achieved": round(d["roofline"]["achieved"], 1),
                              "iteration_gbps": d.get("iteration_gbps"), "relres": d["check"]["relres"]}),
                  flush=True)


if __name__ == "__main__":
    main()
