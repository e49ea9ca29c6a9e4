"""Order-preserving str <-> byte mapping for the reference's str-based API.

The reference works on Python str (code points) and the corpus loader reads
latin-1 (utils/data_loader.py:4), so texts whose code points are all < 256 map
1:1 to bytes.  A text with other code points but at most 256 distinct ones is
remapped densely in sorted order (the same order csa/wavelet_tree.py:68 uses),
which leaves every suffix comparison — hence SA, BWT order, C and ranks — intact.
"""
from __future__ import annotations


class TextCodec:
    def __init__(self, text: str):
        try:
            text.encode("latin-1")
            self.identity = True
            self.to_byte = None
            self.from_byte = None
        except UnicodeEncodeError:
            syms = sorted(set(text))
            if len(syms) > 256:
                raise ValueError("text has more than 256 distinct symbols; the GPU index works on bytes")
            self.identity = False
            self.to_byte = {ch: i for i, ch in enumerate(syms)}
            self.from_byte = "".join(syms)

    def encode_text(self, s: str) -> bytes:
        if self.identity:
            return s.encode("latin-1")
        tb = self.to_byte
        return bytes(tb[ch] for ch in s)

    def encode_pattern(self, s: str) -> bytes | None:
        """Bytes of a query, or None when it holds a symbol the text cannot contain
        (such a pattern never matches: find_range -> (-1, -1))."""
        if self.identity:
            try:
                return s.encode("latin-1")
            except UnicodeEncodeError:
                return None
        tb = self.to_byte
        out = bytearray()
        for ch in s:
            b = tb.get(ch)
            if b is None:
                return None
            out.append(b)
        return bytes(out)

    def encode_symbol(self, ch: str) -> int | None:
        b = self.encode_pattern(ch)
        return b[0] if b is not None and len(b) == 1 else None

    def decode(self, b: bytes) -> str:
        if self.identity:
            return b.decode("latin-1")
        fb = self.from_byte
        return "".join(fb[x] for x in b)
