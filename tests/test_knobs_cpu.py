"""The environment-knob surface stays small and documented: every ``MTA_*`` name the framework reads (Python,
HIP / C++ sources, bench.py / train.py / test.py) appears in the knob table of docs/ARCHITECTURE.md, and there are at
most 40 of them (the negative-result A/B paths were pruned; new ones need a table row and a test)."""
import re
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PAT = re.compile(r"\bMTA_[A-Z0-9_]+\b")


def _knobs():
    names = set()
    files = list((REPO / "masters_thesis_amd").rglob("*.py")) + list((REPO / "csrc").glob("*.hip"))
    files += list((REPO / "csrc").glob("*.h")) + list((REPO / "csrc").glob("*.cpp"))
    files += [REPO / f for f in ("bench.py", "train.py", "test.py", "__graft_entry__.py")]
    for f in files:
        names |= set(PAT.findall(f.read_text(errors="replace")))
    return names


def test_knob_count_and_documentation():
    names = _knobs()
    assert len(names) <= 40, sorted(names)
    doc = (REPO / "docs" / "ARCHITECTURE.md").read_text()
    table = doc[doc.index("## Environment knobs"):]
    missing = sorted(n for n in names if n not in table)
    assert not missing, f"undocumented knobs (add a row to the table in docs/ARCHITECTURE.md): {missing}"
