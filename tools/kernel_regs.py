"""VGPR / SGPR / scratch / LDS of each kernel in a hipcc --save-temps gfx950 assembly file (the
metadata entries; diagnostic for occupancy).  usage: python tools/kernel_regs.py FILE.s [NAME_SUBSTR ...]"""
import re
import sys


def entries(text):
    meta = text[text.find("amdhsa.kernels:"):]
    for blk in re.split(r"\n  - ", meta)[1:]:
        d = dict(re.findall(r"\.(name|vgpr_count|sgpr_count|private_segment_fixed_size|group_segment_fixed_size|"
                            r"vgpr_spill_count|agpr_count):\s+(\S+)", blk))
        if "name" in d:
            yield d


if __name__ == "__main__":
    s = open(sys.argv[1]).read()
    keys = sys.argv[2:]
    for d in entries(s):
        if not keys or any(k in d["name"] for k in keys):
            print(f"{d['name'][:60]:60s} vgpr {d.get('vgpr_count')} agpr {d.get('agpr_count')} sgpr {d.get('sgpr_count')} "
                  f"scratch {d.get('private_segment_fixed_size')} lds {d.get('group_segment_fixed_size')} "
                  f"vspill {d.get('vgpr_spill_count')}")
