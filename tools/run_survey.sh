#!/bin/bash
# Every call kind on seven object shapes (DESIGN.md §5's survey table): the shipped
# library alone, tools/ab_same.py over ab_bench's survey grid, >= 100 ms per cell, 2
# rounds, whole-line output rows (BatchEngine's default) and the bounded calls with
# their rows back to back (`bound` rows per stripe, as bench.py's sweep).
# tools/survey_table.py makes the table.  Usage: tools/run_survey.sh > log
set -o pipefail
WL=$(python3 -c "
import sys; sys.path.insert(0, 'tools')
from ab_bench import SURVEY_MODES, _SURVEY_SHAPES
print(','.join(f'{s}_{m}' + ('@dense' if m in ('rec1pb_out', 'rec2pb_out') else '') for s in _SURVEY_SHAPES for m in SURVEY_MODES))")
timeout -k 10 900 python3 tools/ab_same.py --variants shipped --workloads "$WL" --rounds 2 --out-pad
