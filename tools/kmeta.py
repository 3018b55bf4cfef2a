"""Register / LDS / scratch figures of kernels from a hipcc -S device assembly.
usage: python tools/kmeta.py file.s [name-substring ...]"""
import re
import sys

s = open(sys.argv[1]).read()
md = s[s.find("amdhsa.kernels:"):]
ents = re.split(r"\n  - \.", md)[1:]
for e in ents:
    e = "." + e
    name = re.search(r"\.name:\s+(\S+)", e)
    if not name or (len(sys.argv) > 2 and not any(k in name.group(1) for k in sys.argv[2:])):
        continue
    get = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, e) or [None, "?"])[1]  # noqa: E731
    print(f"{name.group(1)[:70]:70s} vgpr {get('vgpr_count'):>4} agpr {get('agpr_count'):>4} sgpr {get('sgpr_count'):>4} "
          f"lds {get('group_segment_fixed_size'):>7} scratch {get('private_segment_fixed_size'):>5} "
          f"vspill {get('vgpr_spill_count')} sspill {get('sgpr_spill_count')}")
