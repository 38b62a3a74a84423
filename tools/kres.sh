#!/bin/bash
# Register / LDS / spill usage of the kernels of one translation unit (gfx950), from the compiler's
# resource-usage remarks:  tools/kres.sh lif_layers.hip [kernel-name-regex]
set -u
F=${1:-lif_layers.hip}; PAT=${2:-.}
cd snn_event-based_optical_flow_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -I../../include -I. \
  --cuda-device-only -c $F -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c "
import re,sys
pat=re.compile(sys.argv[1]); cur=None; rows=[]
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur={'name':m.group(1)}; rows.append(cur); continue
    for k in ('VGPRs','AGPRs','ScratchSize','Occupancy','LDS Size','VGPRs Spill'):
        m=re.search(r'remark:\s+'+k+r'(?: \[[^\]]*\])?: (\d+)',l)
        if m and cur is not None and k not in cur: cur[k]=int(m.group(1))
for r in rows:
    if pat.search(r['name']): print(r.get('VGPRs'),r.get('AGPRs'),'spill',r.get('VGPRs Spill'),'scratch',r.get('ScratchSize'),'occ',r.get('Occupancy'),'lds',r.get('LDS Size'),r['name'][:110])
" "$PAT"
