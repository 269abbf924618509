"""Build libppo_engine.so for gfx950 with hipcc (in-tree, so the .so travels with the repo).

Each source compiles to an object in parallel (one hipcc per file), then one link step.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = ["csrc/scan_kernels.hip", "csrc/mlp_engine.hip", "csrc/fused_update.hip",
           "csrc/fused_policy.hip", "csrc/bilstm.hip", "csrc/host_rollout.hip",
           "csrc/cnn_engine.hip", "csrc/gemm_ops_fwd_nk.hip", "csrc/gemm_ops_fwd_kn.hip",
           "csrc/gemm_ops_dx.hip", "csrc/gemm_ops_wgrad.hip", "csrc/wide_gemm.hip",
           "csrc/wide_engine.hip", "csrc/comm.hip"]
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-Wall", "-Wno-unused-result"]


def build_host_env(verbose: bool = True) -> str:
    """libppo_hostenv.so: the host physics pool workers' per-slice dynamics (plain C, gcc) and the
    PPO_SEGV_MAPS crash diagnostics (csrc/host/crash_maps.c)."""
    out = os.path.join(HERE, "libppo_hostenv.so")
    srcs = [os.path.join(HERE, "csrc", "host", f) for f in ("synthetic_physics.c", "crash_maps.c")]
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(s) for s in srcs):
        return out
    cmd = [os.environ.get("CC", "gcc"), "-O3", "-ffp-contract=off", "-fPIC", "-shared",
           "-o", out + ".tmp", *srcs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=HERE)
    os.replace(out + ".tmp", out)
    return out


def _object_deps(obj: str, headers: list) -> list:
    """The headers an object was compiled from (its -MMD file), or every header if unknown."""
    dep = obj + ".d"
    if not os.path.exists(dep):
        return headers
    with open(dep) as f:
        words = f.read().replace("\\\n", " ").split()
    files = [w for w in words if not w.endswith(":") and w.endswith(".h")]
    if any(not os.path.exists(f) for f in files):
        return headers
    return files


def build_library(verbose: bool = True) -> str:
    build_host_env(verbose)
    out = os.path.join(HERE, "libppo_engine.so")
    srcs = [os.path.join(HERE, s) for s in SOURCES]
    deps = srcs + glob.glob(os.path.join(HERE, "csrc", "*.h")) + \
        [os.path.join(ROOT, "include", "ppo_engine.h")]
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs, procs = [], []
    headers = [d for d in deps if d.endswith(".h")]
    for src in srcs:
        obj = os.path.join(HERE, "build", os.path.basename(src) + ".o")
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        objs.append(obj)
        if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d)
                                       for d in [src] + _object_deps(obj, headers)):
            continue  # object up to date (per-source incremental rebuild)
        cmd = [hipcc, *FLAGS, "-I", os.path.join(ROOT, "include"), "-MMD", "-MF", obj + ".d",
               "-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd, cwd=HERE)))
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    link = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.run(link, check=True, cwd=HERE)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_library())
