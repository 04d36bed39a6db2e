"""INTEGRATION.md §11 cites include/qba.h by line: every entry point is in
the index, and each row's line range covers the declarations it names."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _decl_lines():
    pos = {}
    for i, line in enumerate((ROOT / "include" / "qba.h").read_text().split("\n"), 1):
        m = re.search(r"QBA_API\s+[\w\s\*]+?\b(qba_\w+)\s*\(", line)
        if m:
            pos[m.group(1)] = i
    return pos


def test_integration_index_cites_qba_h_lines():
    pos = _decl_lines()
    txt = (ROOT / "INTEGRATION.md").read_text()
    index = txt[txt.index("## 11. Entry-point index"):]
    assert set(re.findall(r"`(qba_\w+)`", index)) >= set(pos)
    for row in re.finditer(r"^\| (`qba_[^|]*)\((\d+)(?:-(\d+))?\) \|", index, re.M):
        a, b = int(row.group(2)), int(row.group(3) or row.group(2))
        for name in re.findall(r"`(qba_\w+)`", row.group(1)):
            if name in pos:
                assert a <= pos[name] <= b, (name, pos[name], (a, b))
