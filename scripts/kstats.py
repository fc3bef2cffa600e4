"""VGPR / AGPR / spill counts of every kernel in one .hip file (gfx950), from the code-object metadata.
usage: python scripts/kstats.py pyaceqd_amd/csrc/pt_sweep.hip [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

src = os.path.abspath(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = tempfile.mkdtemp()
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip", "-c", src,
                       "-o", os.path.join(d, "k.o"), "-save-temps"], cwd=d, stdout=subprocess.DEVNULL,
                      stderr=subprocess.DEVNULL)
s = open([os.path.join(d, f) for f in os.listdir(d) if f.endswith("gfx950.s")][0]).read()
meta = s[s.index("amdhsa.kernels:"):]
for blk in meta.split("  - .agpr_count:")[1:]:
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
    name = g("name")
    if flt in name:
        short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)[:60]
        print(f"{short:60s} vgpr {g('vgpr_count'):>4s} agpr {blk.split()[0]:>4s} spill {g('vgpr_spill_count'):>3s} "
              f"lds {g('group_segment_fixed_size')}")
