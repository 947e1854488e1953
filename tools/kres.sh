#!/bin/bash
# Register / spill report of every k_render instantiation in a kernels.hip (default: the tree's):
#   tools/kres.sh [path/to/kernels.hip]
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=${1:-$HERE/../yet-another-raytracer_amd/csrc/kernels.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -I"$HERE/../build/gen" ${KDEFS:-} \
  --cuda-device-only -c -o /dev/null "$SRC" -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None; rows = {}
for line in sys.stdin:
    m = re.search(r"remark: +(.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1)
    if t.startswith("Function Name:"): cur = t.split(":", 1)[1].strip(); rows[cur] = {}; continue
    k, _, v = t.partition(":")
    if cur and k.strip() in ("VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]"): rows[cur][k.strip()] = v.strip()
for n in sorted(rows):
    if "k_render" in n or "k_wf" in n: print(n.replace("_ZN8yart_dev8k_renderI", "k_render<").split("EEv")[0], rows[n])
'
