"""Register / LDS / scratch use per kernel from a device asm file (hipcc --cuda-device-only -S): kstats.py FILE.s [substr].
Analysis aid only."""
import re
import sys

import yaml

t = open(sys.argv[1]).read()
meta = t[t.index(".amdgpu_metadata") + len(".amdgpu_metadata"):t.index(".end_amdgpu_metadata")].replace("\t", " ")
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for k in yaml.safe_load(meta)["amdhsa.kernels"]:
    if sub in k[".name"]:
        print(f"vgpr {k['.vgpr_count']:4d} agpr {k.get('.agpr_count', 0):3d} spill {k.get('.vgpr_spill_count', 0):3d} "
              f"lds {k['.group_segment_fixed_size']:6d} scratch {k['.private_segment_fixed_size']:5d}  {k['.name'][:90]}")
