"""Build the in-tree gfx950 engine ``leanfe_amd/liblfe_hip.so`` with hipcc.

    python -m leanfe_amd.build            # incremental (by content hash)
    python -m leanfe_amd.build --force    # rebuild everything

The shared library is written in-tree so it travels to the GPU box with the
repository snapshot (it is git-ignored, not gpurun-ignored).

Incremental by content, not by timestamp: every object is rebuilt when the hash of its
source, the shared headers and the compiler flags differs from the one recorded beside it
(``_obj/<name>.o.sha``), and the library embeds the hash of all sources
(``lfe_build_hash()``).  ``source_hash()`` is what the checked-out sources hash to;
``_lib.load_library`` refuses a library whose embedded hash differs, so a stale build
can never run silently.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
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

SOURCES = ["lfe_capi.hip", "lfe_prep.hip", "lfe_sweep.hip", "lfe_fast.hip", "lfe_iter.hip", "lfe_dense.hip", "lfe_dense3.hip", "lfe_seg.hip", "lfe_gram.hip", "lfe_cluster.hip", "lfe_keys.hip", "lfe_compress.hip", "lfe_synth.hip", "lfe_shard.hip", "lfe_stream.hip", "lfe_wide.hip", "lfe_fit.hip"]
HEADERS = ["lfe_internal.h", os.path.join("..", "..", "include", "leanfe_hip.h")]

CFLAGS = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
          "-fno-gpu-rdc", "-Wall", "-Wno-unused-result", "-Wno-unused-value", f"-I{ROCM}/include"]
LDFLAGS = ["-shared", f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]
STAMP_MARK = "LFE_SRC_HASH="


def _read(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


def _object_hash(src: str) -> str:
    h = hashlib.sha256()
    h.update(" ".join(CFLAGS).encode())
    for p in [os.path.join(CSRC, src)] + [os.path.join(CSRC, x) for x in HEADERS]:
        h.update(b"\0" + os.path.basename(p).encode() + b"\0" + _read(p))
    return h.hexdigest()


def source_hash() -> str:
    """Hash of every engine source, header and flag: what the library must embed."""
    h = hashlib.sha256()
    for src in SOURCES:
        h.update(_object_hash(src).encode())
    h.update(" ".join(LDFLAGS).encode())
    return h.hexdigest()[:32]


def library_hash(path: str = LIB) -> str | None:
    """The hash embedded in a built library (read from its bytes: nothing is loaded)."""
    try:
        data = _read(path)
    except OSError:
        return None
    i = data.find(STAMP_MARK.encode())
    if i < 0:
        return None
    j = i + len(STAMP_MARK)
    return data[j:j + 32].decode(errors="replace")


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, src.replace(".hip", ".o"))
    stamp = obj + ".sha"
    want = _object_hash(src)
    have = _read(stamp).decode().strip() if os.path.exists(stamp) else None
    if force or have != want or not os.path.exists(obj):
        cmd = [HIPCC, *CFLAGS, "-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        if r.stderr.strip():
            sys.stderr.write(r.stderr)
        with open(stamp, "w") as f:
            f.write(want + "\n")
    return obj


def _stamp_object(digest: str) -> str:
    """A host-only object exporting lfe_build_hash() (the marker keeps the hash findable in the .so)."""
    src = os.path.join(OBJ, "lfe_stamp.cpp")
    obj = os.path.join(OBJ, "lfe_stamp.o")
    with open(src, "w") as f:
        f.write('extern "C" const char* lfe_build_hash(void) {\n'
                f'  static const char k[] = "{STAMP_MARK}{digest}";\n'
                f'  return k + {len(STAMP_MARK)};\n}}\n')
    r = subprocess.run(["g++", "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"stamp compile failed:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    digest = source_hash()
    if force or library_hash() != digest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", *objs, _stamp_object(digest), "-o", LIB, *LDFLAGS]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB} (sources {digest})")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    build(force=ap.parse_args().force)
