"""VGPR / spill / LDS of the kernels of the built library whose mangled name contains the argument."""
import re
import subprocess
import sys
import tempfile

LL = "/opt/rocm/lib/llvm/bin"
tmp = tempfile.mkdtemp()
obj = sys.argv[2] if len(sys.argv) > 2 else "of_dis_amd/csrc/build/ofdis_kernels.o"
subprocess.run([f"{LL}/llvm-objcopy", f"--dump-section=.hip_fatbin={tmp}/f", obj], check=True)
subprocess.run([f"{LL}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={tmp}/f",
                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={tmp}/k.co"], check=True)
out = subprocess.run([f"{LL}/llvm-readelf", "--notes", f"{tmp}/k.co"], capture_output=True, text=True).stdout
for blk in out.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if sys.argv[1] in name:
        g = lambda k: re.search(rf"\.{k}:\s+(\d+)", blk).group(1)
        print(f"{name[:90]:90s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>4} lds {g('group_segment_fixed_size')}")
