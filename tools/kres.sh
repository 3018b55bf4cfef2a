#!/bin/bash
# per-kernel VGPR / occupancy / scratch of the HIP library (compile only)
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I include ${@} mast3r-slam-ysh_amd/csrc/m3s_gn.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys,re,subprocess
cur=None; rows={}
for l in sys.stdin:
    m=re.search(r"Function Name: (\S+)",l)
    if m: cur=subprocess.run(["c++filt"],input=m.group(1),capture_output=True,text=True).stdout.strip().replace("(anonymous namespace)::",""); rows[cur]={}; continue
    for k in ("VGPRs","AGPRs","ScratchSize \[bytes/lane\]","Occupancy \[waves/SIMD\]","LDS Size \[bytes/block\]"):
        m=re.search(k+r": (\d+)",l)
        if m and cur: rows[cur][k.split()[0]]=m.group(1)
for k,v in rows.items():
    if "linearize" in k or "llt" in k or "chol" in k: print(v.get("VGPRs"),v.get("AGPRs"),v.get("ScratchSize"),v.get("Occupancy"),v.get("LDS"),k[:110])
'
