# VGPR / spill counts of the gfx950 kernels in one built object whose mangled name contains PATTERN.
# usage: bash tools/isa_regs.sh conv_gemm PATTERN   (reads multimodal-organ-segmentation_amd/csrc/build/<src>.hip.o)
set -e
SRC=${1:-conv_gemm}; PAT=${2:-.}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/isa.XXXX)
cp "$R/multimodal-organ-segmentation_amd/csrc/build/$SRC.hip.o" "$T/k.o"
(cd "$T" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading k.o > /dev/null 2>&1)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/k.o.0.hipv4-amdgcn-amd-amdhsa--gfx950" > "$T/notes.txt"
python3 - "$T/notes.txt" "$PAT" <<'EOF'
import re, sys
t = open(sys.argv[1]).read()
for blk in t.split('  - .agpr_count')[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk).group(1)
    if not re.search(sys.argv[2], name):
        continue
    v = re.search(r'\.vgpr_count:\s+(\d+)', blk).group(1)
    s = re.search(r'\.vgpr_spill_count:\s+(\d+)', blk).group(1)
    print(f'{v:>4} vgpr {s:>3} spill  {name}')
EOF
rm -rf "$T"
