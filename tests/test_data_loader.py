"""Corpus ingest (utils/data_loader.py:3-7 of the reference): gzip, latin-1, text-mode newlines,
`size_limit` in characters, and the hand-off of the loaded str to the byte codec the GPU index
uses.  CPU only."""
import gzip

import pytest

from hkcsa import TextCodec
from oracle import oracle
from utils.data_loader import load_text


def _write(tmp_path, name, raw: bytes):
    p = tmp_path / name
    with gzip.open(p, "wb") as fh:
        fh.write(raw)
    return str(p)


def test_latin1_bytes_round_trip(tmp_path):
    raw = bytes(range(1, 256)) * 3   # every byte but NUL; 0x80-0xFF are latin-1 letters, not UTF-8
    raw = raw.replace(b"\r", b"")    # (\r is covered by the newline test)
    p = _write(tmp_path, "all.gz", raw)
    s = load_text(p)
    assert s == raw.decode("latin-1")
    assert TextCodec(s).identity
    assert TextCodec(s).encode_text(s) == raw


def test_crlf_and_cr_are_universal_newlines(tmp_path):
    p = _write(tmp_path, "nl.gz", b"ACGT\r\nACGA\rTTT\n")
    s = load_text(p)
    assert s == "ACGT\nACGA\nTTT\n"   # text mode: \r\n and \r read as \n, as the reference's loader
    assert "\r" not in s


@pytest.mark.parametrize("limit", [1, 5, 6, 7, 100])
def test_size_limit_counts_characters(tmp_path, limit):
    raw = b"AC\r\nGT\xe9\xe8" * 4
    p = _write(tmp_path, "lim.gz", raw)
    full = raw.decode("latin-1").replace("\r\n", "\n")
    assert load_text(p, size_limit=limit) == full[:limit]


@pytest.mark.parametrize("limit", [None, 0])
def test_no_limit_reads_everything(tmp_path, limit):
    raw = b"GATTACA" * 1000
    p = _write(tmp_path, "full.gz", raw)
    assert load_text(p, size_limit=limit) == raw.decode("latin-1")   # 0 is falsy: whole file


def test_empty_file(tmp_path):
    p = _write(tmp_path, "empty.gz", b"")
    assert load_text(p) == ""
    assert load_text(p, size_limit=10) == ""


def test_not_gzip_raises(tmp_path):
    p = tmp_path / "plain.txt"
    p.write_bytes(b"ACGT")
    with pytest.raises(OSError):
        load_text(str(p))


def test_loaded_text_feeds_the_index_bytes(tmp_path):
    # the loaded corpus + '$' is what the drop-in builds on: its bytes' suffix array (oracle) is the
    # reference's SA of the str (latin-1 keeps code-point order)
    raw = b"mississippi\r\n\xe9t\xe9"
    p = _write(tmp_path, "corpus.gz", raw)
    s = load_text(p) + "$"
    b = TextCodec(s).encode_text(s)
    ref = sorted(range(len(s)), key=lambda i: s[i:])
    assert list(oracle.suffix_array(b)) == ref
