"""Drop-in for the reference's utils/data_loader.py:3-7 (corpus ingest).

Reads a gzip file as latin-1 text (universal newlines, as text mode does),
optionally only the first `size_limit` characters.
"""
from __future__ import annotations

import gzip


def load_text(path, size_limit=None):
    with gzip.open(path, "rt", encoding="latin-1") as fh:
        return fh.read(size_limit) if size_limit else fh.read()
