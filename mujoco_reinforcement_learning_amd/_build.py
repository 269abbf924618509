"""Build libppo_engine.so for gfx950 with hipcc (in-tree, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = ["csrc/scan_kernels.hip", "csrc/mlp_engine.hip"]
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-Wall", "-Wno-unused-result"]


def build_library(verbose: bool = True) -> str:
    out = os.path.join(HERE, "libppo_engine.so")
    srcs = [os.path.join(HERE, s) for s in SOURCES]
    deps = srcs + [os.path.join(HERE, "csrc", "common.h"),
                   os.path.join(ROOT, "include", "ppo_engine.h")]
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *FLAGS, "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp", *srcs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=HERE)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_library())
