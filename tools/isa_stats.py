"""Per-kernel static ISA statistics of a hipcc -S device assembly file:
instruction counts by class, VGPR / SGPR / LDS / scratch.
    python tools/isa_stats.py file.s [name-substring ...]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().splitlines()
want = sys.argv[2:]
kernels = {}
cur = None
for line in src:
    m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
    if m and not line.startswith("\t"):
        cur = m.group(1)
        kernels[cur] = Counter()
        continue
    if cur is None:
        continue
    if line.startswith("\t.section") or line.startswith("\t.size\t" + cur):
        cur = None
        continue
    t = line.strip()
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    op = t.split()[0]
    cls = ("v_" if op.startswith("v_") else "s_" if op.startswith("s_") else
           "ds_" if op.startswith("ds_") else "global_" if op.startswith(("global_", "buffer_", "flat_")) else "other")
    if op.startswith(("s_cbranch", "s_branch")):
        cls = "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        cls = "smem"
    kernels[cur][cls] += 1
    kernels[cur]["total"] += 1
meta = {}
for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n){0,40}?", "\n".join(src)):
    pass
text = "\n".join(src)
for k, c in kernels.items():
    if want and not any(w in k for w in want):
        continue
    if c["total"] < 20:
        continue
    blk = re.search(r"\.symbol:\s+" + re.escape(k) + r"\.kd(.*?)(?:\n\s+- \.|\n\.end_amdgpu_metadata)", text, re.S)
    info = {}
    if blk:
        for key in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size",
                    "vgpr_spill_count", "sgpr_spill_count"):
            mm = re.search(r"\." + key + r":\s+(\d+)", blk.group(1))
            if mm:
                info[key] = int(mm.group(1))
    short = re.sub(r"^_ZN3vts\d*_GLOBAL__N_1", "", k)[:60]
    print(short, dict(c), info)
