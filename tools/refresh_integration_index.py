#!/usr/bin/env python3
"""Rewrite the qba.h line ranges cited in INTEGRATION.md section 11 from the
header as it stands (tests/test_docs_index.py checks them)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
pos = {}
for i, line in enumerate((ROOT / "include" / "qba.h").read_text().split("\n"), 1):
    m = re.search(r"QBA_API\s+[\w\s\*]+?\b(qba_\w+)\s*\(", line)
    if m:
        pos[m.group(1)] = i
path = ROOT / "INTEGRATION.md"
head, idx = path.read_text().split("## 11. Entry-point index", 1)


def fix(m):
    lines = [pos[n] for n in re.findall(r"`(qba_\w+)`", m.group(1)) if n in pos]
    a, b = min(lines), max(lines)
    return f"| {m.group(1)}({a})" if a == b else f"| {m.group(1)}({a}-{b})"


idx = re.sub(r"^\| (`qba_[^|]*)\((\d+)(?:-(\d+))?\)", fix, idx, flags=re.M)
path.write_text(head + "## 11. Entry-point index" + idx)
