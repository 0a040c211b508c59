"""Minimal .xlsx reader for the reference's label / process-parameter workbooks.

The reference reads ``Excel/Processed_Circle_test.xlsx`` and ``Excel/Process_parameters.xlsx``
with ``pandas.read_excel`` (``models/CvT(Par).py:60-64``), which needs openpyxl (not in this
image).  This reads the first worksheet straight from the OOXML zip (shared strings, inline
strings, numbers, booleans) and returns it the way the reference indexes it: a header row
(pandas naming: an empty header cell at 0-based column i is ``"Unnamed: i"``) and data rows
addressed by position, data row k = worksheet row k + 2 (``DataFrame.loc[k, name]``).
"""
from __future__ import annotations

import math
import re
import zipfile
import xml.etree.ElementTree as ET
from typing import Any, Dict, List, Optional

_NS = "{http://schemas.openxmlformats.org/spreadsheetml/2006/main}"
_REF = re.compile(r"([A-Z]+)(\d+)")


def _col_index(letters: str) -> int:
    n = 0
    for ch in letters:
        n = n * 26 + (ord(ch) - 64)
    return n - 1


def _text(node) -> str:
    return "".join(t.text or "" for t in node.iter(_NS + "t"))


class Sheet:
    """``header`` (list of column names) and ``cell(row, name)`` -> float | str | bool | nan."""

    def __init__(self, header: List[str], rows: Dict[int, Dict[int, Any]], nrows: int):
        self.header = header
        self._col = {h: i for i, h in enumerate(header)}
        self._rows = rows
        self.nrows = nrows

    def cell(self, row: int, name: str) -> Any:
        if name not in self._col:
            raise KeyError(f"column {name!r} not in {self.header}")
        if not 0 <= row < self.nrows:
            raise KeyError(f"row {row} out of range [0, {self.nrows})")
        v = self._rows.get(row, {}).get(self._col[name])
        return math.nan if v is None else v

    def column(self, name: str) -> List[Any]:
        return [self.cell(r, name) for r in range(self.nrows)]


def read_xlsx(path: str) -> Sheet:
    z = zipfile.ZipFile(path)
    shared: List[str] = []
    if "xl/sharedStrings.xml" in z.namelist():
        root = ET.fromstring(z.read("xl/sharedStrings.xml"))
        shared = [_text(si) for si in root.iter(_NS + "si")]
    root = ET.fromstring(z.read("xl/worksheets/sheet1.xml"))
    cells: Dict[int, Dict[int, Any]] = {}
    max_row, max_col = 0, -1
    for row in root.iter(_NS + "row"):
        for c in row.iter(_NS + "c"):
            m = _REF.fullmatch(c.get("r", ""))
            if not m:
                continue
            col, r = _col_index(m.group(1)), int(m.group(2))
            t = c.get("t")
            v = c.find(_NS + "v")
            val: Optional[Any] = None
            if t == "inlineStr":
                is_ = c.find(_NS + "is")
                val = _text(is_) if is_ is not None else None
                val = val if val else None
            elif v is not None and v.text is not None:
                if t == "s":
                    val = shared[int(v.text)]
                elif t in ("str", "e"):
                    val = v.text
                elif t == "b":
                    val = v.text.strip() == "1"
                else:
                    val = float(v.text)
            if val is None:
                continue
            cells.setdefault(r, {})[col] = val
            max_row, max_col = max(max_row, r), max(max_col, col)
    hdr_cells = cells.get(1, {})
    header = [str(hdr_cells[i]) if i in hdr_cells else f"Unnamed: {i}" for i in range(max_col + 1)]
    rows = {r - 2: v for r, v in cells.items() if r >= 2}
    return Sheet(header, rows, max(0, max_row - 1))
