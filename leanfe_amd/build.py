"""Build the in-tree gfx950 engine ``leanfe_amd/liblfe_hip.so`` with hipcc.

    python -m leanfe_amd.build            # incremental
    python -m leanfe_amd.build --force    # rebuild everything

The shared library is written in-tree so it travels to the GPU box with the
repository snapshot (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "csrc", "_obj")
LIB = os.path.join(HERE, "liblfe_hip.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = "gfx950"

SOURCES = ["lfe_capi.hip", "lfe_prep.hip", "lfe_sweep.hip", "lfe_fast.hip", "lfe_iter.hip", "lfe_seg.hip", "lfe_gram.hip", "lfe_cluster.hip", "lfe_keys.hip", "lfe_compress.hip", "lfe_synth.hip"]
HEADERS = ["lfe_internal.h", os.path.join("..", "..", "include", "leanfe_hip.h")]

CFLAGS = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
          "-fno-gpu-rdc", "-Wall", "-Wno-unused-result", "-Wno-unused-value", f"-I{ROCM}/include"]
LDFLAGS = ["-shared", f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, src.replace(".hip", ".o"))
    deps = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in HEADERS]
    if force or _stale(obj, deps):
        cmd = [HIPCC, *CFLAGS, "-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        if r.stderr.strip():
            sys.stderr.write(r.stderr)
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", *objs, "-o", LIB, *LDFLAGS]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    build(force=ap.parse_args().force)
