"""Markdown table of a survey run (tools/ab_same.py over ab_bench's survey grid):
rows = object shapes, columns = call kinds, cells = fraction of 8 TB/s (kernel).
Usage: python tools/survey_table.py profiles/<tag>_survey.log"""
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from ab_bench import SURVEY_MODES, _SURVEY_SHAPES  # noqa: E402

LABEL = {"enc": "encode", "ver": "scrub", "rec2u": "2 lost, one pattern, in place",
         "rec2u_out": "2 lost, one pattern", "rec2p": "2 lost per stripe, in place",
         "rec1pb_out": "1 lost, bound 1", "rec2pb_out": "2 lost, bound 2", "rec2p_out": "2 lost, no bound",
         "recmix_out": "0..m lost (scan)"}
SHAPE = {"rs42_4K": "RS(4+2) 4 KiB", "rs42_64K": "RS(4+2) 64 KiB", "rs42_1M": "RS(4+2) 1 MiB",
         "rs84_64K": "RS(8+4) 64 KiB", "rs104_64K": "RS(10+4) 64 KiB", "rs104_80K": "RS(10+4) 80 KiB",
         "rs63_48K": "RS(6+3) 48 KiB"}


def main():
    got = {}
    for ln in open(sys.argv[1]):
        m = re.match(r"(\S+)\s+\S+\s+median\s+([\d.]+)%", ln)
        if m:
            got[m.group(1).split("@")[0]] = float(m.group(2)) / 100  # "@dense": the output-row layout
    print("| shape | " + " | ".join(LABEL[md] for md in SURVEY_MODES) + " |")
    print("|---" * (len(SURVEY_MODES) + 1) + "|")
    for sh in _SURVEY_SHAPES:
        cells = [f"{got[f'{sh}_{md}']:.2f}" if f"{sh}_{md}" in got else "—" for md in SURVEY_MODES]
        print(f"| {SHAPE[sh]} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
