"""Build an experiment variant of the engine with extra preprocessor flags, for same-box A/B
(LEANFE_HIP_LIB selects it):  python tools/build_variant.py tools/var/old.so -DLFE_OLD_STAGING
The in-tree objects are untouched; the variant links its own objects under /tmp."""
import concurrent.futures as cf
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from leanfe_amd import build as B  # noqa: E402

out, defs = sys.argv[1], sys.argv[2:]
tmp = tempfile.mkdtemp()


def comp(src):
    obj = os.path.join(tmp, src.replace(".hip", ".o"))
    r = subprocess.run([B.HIPCC, *B.CFLAGS, "-w", *defs, "-c", os.path.join(B.CSRC, src), "-o", obj],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    return obj


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(comp, B.SOURCES))
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", *objs, B._stamp_object("variant" + "0" * 25), "-o", out,
                    *B.LDFLAGS], capture_output=True, text=True)
if r.returncode:
    raise SystemExit(r.stderr)
print("built", out, defs)
