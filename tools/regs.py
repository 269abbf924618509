"""Per-kernel register / spill summary from an amdgcn .s file (AMDHSA metadata block)."""
import re
import sys

txt = open(sys.argv[1]).read()
meta = txt[txt.find("amdhsa.kernels:"):]
for blk in meta.split("\n  - ")[1:]:
    def g(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"
    name = g("name")
    if len(sys.argv) > 2 and sys.argv[2] not in name:
        continue
    print(f"vgpr {g('vgpr_count'):>4} vspill {g('vgpr_spill_count'):>3} sgpr {g('sgpr_count'):>4} "
          f"sspill {g('sgpr_spill_count'):>3} lds {g('group_segment_fixed_size'):>6}  {name}")
