"""Per-kernel VGPR / spill / LDS / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage."""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "leanfe_amd", "csrc")
files = sys.argv[1:] or ["lfe_prep.hip", "lfe_sweep.hip", "lfe_gram.hip", "lfe_synth.hip"]
for f in files:
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
           "-I/opt/rocm/include", "-c", os.path.join(SRC, f), "-o", "/tmp/_rr.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(.*", "", name)
        print(f"{f:14s} {name[:48]:48s} VGPR={r.get('VGPRs','?'):>4} AGPR={r.get('AGPRs','?'):>3} "
              f"spillV={r.get('VGPRs Spill','?'):>3} spillS={r.get('SGPRs Spill','?'):>3} "
              f"LDS={r.get('LDS Size [bytes/block]','?'):>6} occ={r.get('Occupancy [waves/SIMD]','?')}")
