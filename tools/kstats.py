"""Diagnostics: registers, scratch and LDS of the kernels in a built object (.o of a .hip),
from the code object's metadata notes.  python tools/kstats.py <obj.o> [name-filter]"""
import re
import subprocess
import sys

B = "/opt/rocm/lib/llvm/bin"
obj, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
subprocess.run([f"{B}/llvm-objcopy", "--dump-section=.hip_fatbin=/tmp/_k.fatbin", obj], check=True)
subprocess.run([f"{B}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                "--input=/tmp/_k.fatbin", "--output=/tmp/_k.co", "--unbundle"], check=True)
txt = subprocess.run([f"{B}/llvm-readelf", "--notes", "/tmp/_k.co"], capture_output=True, text=True).stdout
for blk in txt.split("- .agpr_count")[1:]:
    g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
    n = g("name")
    dn = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    if filt not in dn:
        continue
    print(f"priv={g('private_segment_fixed_size'):>5} vgpr={g('vgpr_count'):>3} sgpr={g('sgpr_count'):>3} "
          f"vspill={g('vgpr_spill_count'):>4} lds={g('group_segment_fixed_size'):>6} {dn[:120]}")
