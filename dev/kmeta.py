"""Per-kernel LDS / VGPR / SGPR of a built object (code-object metadata): python dev/kmeta.py [obj] [filter]"""
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin/"
obj = sys.argv[1] if len(sys.argv) > 1 else "cuda.radixsort_amd/build/rsort_kernels.o"
flt = sys.argv[2] if len(sys.argv) > 2 else "rs_scatter"
subprocess.run([LLVM + "llvm-objcopy", "--dump-section=.hip_fatbin=/tmp/_fat.bin", obj], check=True)
subprocess.run([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                "--input=/tmp/_fat.bin", "--output=/tmp/_dev.o"], check=True)
notes = subprocess.run([LLVM + "llvm-readelf", "--notes", "/tmp/_dev.o"], capture_output=True, text=True).stdout
for blk in notes.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if flt not in name:
        continue
    dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    g = lambda k: re.search(rf"\.{k}:\s+(\d+)", blk).group(1)
    print(f"lds={g('group_segment_fixed_size'):>7} vgpr={g('vgpr_count'):>4} sgpr={g('sgpr_count'):>4} spill={g('vgpr_spill_count')} scratch={g('private_segment_fixed_size')}  {dm}")
