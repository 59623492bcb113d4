"""DESIGN.md's result tables are generated from committed profiles
(tools/design_tables.py <tag>, tools/survey_table.py): every generated table row must
appear verbatim in DESIGN.md, so the document cannot drift from the evidence it cites."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _design():
    return open(os.path.join(ROOT, "DESIGN.md")).read()


def _tag():
    m = re.search(r"`tools/design_tables.py (r\d+\w*)`", _design())
    assert m, "DESIGN.md names the tag its tables come from"
    return m.group(1)


def _rows(text):
    return [ln for ln in text.splitlines() if ln.startswith("| ") and not ln.startswith("|---")]


def test_result_tables_match_committed_profiles():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "design_tables.py"), _tag()],
                         capture_output=True, text=True, check=True).stdout
    rows = _rows(out)
    assert len(rows) > 30
    design = _design()
    missing = [r for r in rows if r not in design]
    assert not missing, missing[:5]


def test_survey_table_matches_committed_log():
    m = re.search(r"`profiles/(r\w+_survey\.log)`", _design())
    assert m, "DESIGN.md cites its survey log"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "survey_table.py"),
                          os.path.join(ROOT, "profiles", m.group(1))], capture_output=True, text=True,
                         check=True).stdout
    design = _design()
    missing = [r for r in _rows(out) if r not in design]
    assert not missing, missing[:5]
