"""Order-preserving str <-> byte mapping for the reference's str-based API.

The reference works on Python str (code points) and the corpus loader reads
latin-1 (utils/data_loader.py:4), so texts whose code points are all < 256 map
1:1 to bytes.  A text with other code points but at most 256 distinct ones is
remapped densely in sorted order (the same order csa/wavelet_tree.py:68 uses),
which leaves every suffix comparison — hence SA, BWT order, C and ranks — intact.

Large texts never pass through a per-character Python loop, and the identity case is not copied
at all: on CPython a str stores its code points as one flat array of 1, 2 or 4 bytes each, and
`TextCodec.parts` hands that array to the upload as a read-only numpy view (checked against the str's
own encoding at both ends before it is trusted; any other interpreter or layout takes the plain
`str.encode` copy).  A remap counts the code points of the 2/4-byte array with numpy (a histogram
over the code-point range, in chunks) and maps them through a 256-entry-wide lookup table.
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

_CHUNK = 1 << 24
_ENC = {1: "latin-1", 2: "utf-16-le", 4: "utf-32-le"}


def _layout():
    """(state offset, ascii header, compact header) of CPython's compact str objects, or None."""
    if sys.implementation.name != "cpython" or C.sizeof(C.c_void_p) != 8:
        return None
    ha = sys.getsizeof("") - 1            # PyASCIIObject + the NUL of ""
    hc = sys.getsizeof("\xe9") - 2        # PyCompactUnicodeObject + 1 char + NUL
    lay = (32, ha, hc)                    # state follows refcnt, type, length, hash
    probes = ["", "abc", "\xe9t\xe9", "āb", "\U0001f600x"]
    for s, kind in zip(probes, (1, 1, 1, 2, 4)):
        v = _view(s, lay)
        if v is None or v.itemsize != kind or len(v) != len(s) or \
                (len(s) and v.tobytes() != s.encode(_ENC[kind], "surrogatepass")):
            return None
    return lay


def _view(s: str, lay):
    """Read-only numpy view of the code-point array of str `s` (uint8/16/32), or None."""
    st = C.c_uint32.from_address(id(s) + lay[0]).value
    kind, compact, ascii_ = (st >> 2) & 7, (st >> 5) & 1, (st >> 6) & 1
    if not compact or kind not in (1, 2, 4):
        return None
    n = len(s)
    dt = {1: np.uint8, 2: np.uint16, 4: np.uint32}[kind]
    if n == 0:
        return np.zeros(0, dtype=dt)
    addr = id(s) + (lay[1] if ascii_ else lay[2])
    buf = (C.c_char * (n * kind)).from_address(addr)
    buf._src = s   # the view's base chain (view -> buf -> s) keeps the str, hence its storage, alive
    v = np.frombuffer(buf, dtype=dt)
    v.flags.writeable = False
    return v


_LAYOUT = _layout()


def code_points(s: str) -> np.ndarray:
    """The code points of `s` as a uint8 / uint16 / uint32 array: a zero-copy view of the str's own
    storage on CPython (the view holds a reference to `s`), else an encoded copy."""
    if _LAYOUT is not None:
        v = _view(s, _LAYOUT)
        if v is not None:
            head, tail = s[:16], s[-16:]
            enc = _ENC[v.itemsize]
            if v[:len(head)].tobytes() == head.encode(enc, "surrogatepass") and \
                    v[len(v) - len(tail):].tobytes() == tail.encode(enc, "surrogatepass"):
                return v
    try:
        return np.frombuffer(s.encode("latin-1"), dtype=np.uint8)
    except UnicodeEncodeError:
        return np.frombuffer(s.encode("utf-32-le", "surrogatepass"), dtype=np.uint32)


class TextCodec:
    def __init__(self, text: str, extra: str = ""):
        """Mapping for the symbols of text + extra (the concatenation is never built)."""
        cps = [code_points(text), code_points(extra)]
        if all(c.dtype == np.uint8 for c in cps):
            self.identity = True
            self.syms = None
            self.lut = None
            self.to_byte = None
            return
        top = max(int(c.max()) if len(c) else 0 for c in cps) + 1
        cnt = np.zeros(top, dtype=np.int64)
        for c in cps:
            for a in range(0, len(c), _CHUNK):
                cnt += np.bincount(c[a:a + _CHUNK], minlength=top)
        syms = np.flatnonzero(cnt)
        if len(syms) > 256:
            raise ValueError("text has more than 256 distinct symbols; the GPU index works on bytes")
        self.identity = False
        self.syms = syms.astype(np.uint32)
        self.lut = np.zeros(top, dtype=np.uint8)
        self.lut[syms] = np.arange(len(syms), dtype=np.uint8)
        self.to_byte = {chr(int(c)): i for i, c in enumerate(syms)}

    def parts(self, *texts: str) -> list[np.ndarray]:
        """uint8 arrays whose concatenation is the encoding of texts[0] + texts[1] + ... — views of the
        strs themselves when the mapping is the identity (keep the strs alive while they are used)."""
        out = []
        for t in texts:
            c = code_points(t)
            if self.identity:
                out.append(c)
                continue
            e = np.empty(len(c), dtype=np.uint8)
            for a in range(0, len(c), _CHUNK):
                e[a:a + _CHUNK] = self.lut[c[a:a + _CHUNK]]
            out.append(e)
        return out

    def encode_text(self, s: str) -> bytes:
        if self.identity:
            return s.encode("latin-1")
        return self.parts(s)[0].tobytes()

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

    def decode(self, b) -> str:
        if self.identity:
            return bytes(b).decode("latin-1")
        a = np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray, memoryview)) else \
            np.asarray(b, dtype=np.uint8)
        return self.syms[a].astype("<u4").tobytes().decode("utf-32-le", "surrogatepass")
