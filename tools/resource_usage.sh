#!/bin/bash
# Compact per-kernel resource table (VGPRs, SGPRs, scratch, spills) of one LM translation unit.
# usage: tools/resource_usage.sh [csrc/fmpnp_lm_f32.hip]
cd "$(dirname "$0")/../featuremetric-pnp_amd"
SRC=${1:-csrc/fmpnp_lm_f32.hip}
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -I../include -Icsrc -c "$SRC" -o /tmp/ru.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = {"name": m.group(1)}; rows.append(cur); continue
    m = re.search(r"\s(VGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None: cur[m.group(1)] = int(m.group(2))
for r in rows:
    n = re.sub(r"_ZN5fmpnp9lm_kernelI(\w)Li(\d)ELb(\d)ELb(\d)ELi(\d+)EEEvNS_10LaunchArgsE", r"lm<\1,wps\2,team\3,ratio\4,var\5>", r["name"])
    g = lambda k: r.get(k, 0)
    print("%-40s vgpr %4d sgpr %4d scratch %5d vspill %4d" % (n, g("VGPRs"), g("TotalSGPRs"), g("ScratchSize [bytes/lane]"), g("VGPRs Spill")))
'
