"""VGPR / AGPR / spill / LDS figures of the kernels in a built object whose symbol contains a substring.
Usage: python tools/kreg.py OBJ SUBSTR [SUBSTR2 ...]"""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd", "csrc"))
import isa_check  # noqa: E402


def main():
    notes = []
    isa_check.disasm(sys.argv[1], notes)
    text = notes[0]
    for blk in re.split(r"\n\s*- \.", text):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or not all(s in m.group(1) for s in sys.argv[2:]):
            continue
        f = {k: re.search(rf"\.{k}:\s+(\d+)", blk) for k in ("vgpr_count", "agpr_count", "vgpr_spill_count",
                                                            "group_segment_fixed_size", "sgpr_count")}
        print(" ".join(f"{k}={v.group(1) if v else '-'}" for k, v in f.items()), m.group(1)[:120])


if __name__ == "__main__":
    main()
