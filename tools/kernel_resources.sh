#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy of the product's HIP sources (hipcc -Rpass-analysis), to catch
# register spills and stack frames (a non-inlined device call copies the parameter block to scratch).
cd "$(dirname "$0")/../zeebe_amd/csrc"
for f in ${@:-zb_wave.hip zb_traj.hip zb_serialize.hip zb_aux.hip zb_msg.hip zb_state.hip}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c -o /tmp/kr_$$.o "$f" -Rpass-analysis=kernel-resource-usage 2>&1 |
    grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | paste - - - - |
    sed -E 's/[^ ]*remark: //g; s/\[-Rpass-analysis=kernel-resource-usage\]//g; s/ +/ /g' |
    awk -v f="$f" '{print f ": " $0}'
done
rm -f /tmp/kr_$$.o
