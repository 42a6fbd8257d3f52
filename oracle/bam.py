"""Minimal BAM writer/reader (pure Python, zlib BGZF) -- TEST INFRASTRUCTURE ONLY.

pysam is not installed here (ordinary ModuleNotFoundError).  The region binning of
/root/reference/ont_tcr_consensus/region_split.py:219-333 reads BAM through pysam.AlignmentFile; these helpers
write seeded BAM inputs for the tests and back a pysam.AlignmentFile stand-in (AlignedSegment with the
attributes that function reads: is_unmapped, is_secondary, is_supplementary, is_reverse, reference_name,
reference_length, query_length, query_name, query_sequence, get_forward_sequence()) following the SAM/BAM
specification (BGZF blocks of <= 64 KiB; record: block_size, refID, pos, l_read_name, mapq, bin, n_cigar_op,
flag, l_seq, next_refID, next_pos, tlen, read_name, cigar, 4-bit seq, qual, no tags).
"""
from __future__ import annotations

import gzip
import struct
import zlib

SEQ_CODES = "=ACMGRSVTWYHKDBN"
CIGAR_OPS = "MIDNSHP=X"
_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _bgzf_block(data: bytes) -> bytes:
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = c.compress(data) + c.flush()
    bsize = len(comp) + 25
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    return hdr + comp + struct.pack("<II", zlib.crc32(data) & 0xffffffff, len(data))


def write_bam(path: str, refs: list, records: list, block: int = 60000) -> None:
    """refs: [(name, length)]; records: dicts with name, flag, ref (index or -1), pos, cigar [(op, len)], seq."""
    raw = bytearray(b"BAM\x01")
    text = b"@HD\tVN:1.6\n"
    raw += struct.pack("<i", len(text)) + text + struct.pack("<i", len(refs))
    for name, ln in refs:
        nb = name.encode() + b"\0"
        raw += struct.pack("<i", len(nb)) + nb + struct.pack("<i", ln)
    for r in records:
        name = r["name"].encode() + b"\0"
        seq = r["seq"]
        cig = b"".join(struct.pack("<I", (ln << 4) | CIGAR_OPS.index(op)) for op, ln in r["cigar"])
        codes = [SEQ_CODES.index(ch) for ch in seq]
        packed = bytes(((codes[i] << 4) | (codes[i + 1] if i + 1 < len(codes) else 0)) for i in range(0, len(codes), 2))
        body = struct.pack("<iiBBHHHiiii", r["ref"], r["pos"], len(name), 60, 4680, len(r["cigar"]), r["flag"], len(seq),
                           -1, -1, 0) + name + cig + packed + b"\xff" * len(seq)
        raw += struct.pack("<i", len(body)) + body
    with open(path, "wb") as fh:
        for i in range(0, len(raw), block):
            fh.write(_bgzf_block(bytes(raw[i:i + block])))
        fh.write(_EOF)


_COMP = str.maketrans("ACGTacgtNnXx", "TGCAtgcaNnXx")


class AlignedSegment:
    def __init__(self, refs, ref, pos, flag, name, cigar, seq):
        self._refs, self.reference_id, self.reference_start, self.flag = refs, ref, pos, flag
        self.query_name, self.cigartuples, self.query_sequence = name, cigar, seq

    is_unmapped = property(lambda s: bool(s.flag & 0x4))
    is_secondary = property(lambda s: bool(s.flag & 0x100))
    is_supplementary = property(lambda s: bool(s.flag & 0x800))
    is_reverse = property(lambda s: bool(s.flag & 0x10))
    reference_name = property(lambda s: s._refs[s.reference_id][0] if s.reference_id >= 0 else None)
    query_length = property(lambda s: len(s.query_sequence or ""))

    @property
    def reference_length(self):
        if self.is_unmapped:
            return None
        # pysam: bam_endpos(b) - pos, and htslib's bam_endpos turns a zero reference span (no CIGAR) into 1
        # (reference_end, not reference_length, is the one that is None without a CIGAR)
        return sum(ln for op, ln in (self.cigartuples or ()) if op in (0, 2, 3, 7, 8)) or 1

    def get_forward_sequence(self):
        s = self.query_sequence
        return s[::-1].translate(_COMP) if (s is not None and self.is_reverse) else s


def read_bam(path: str):
    """(refs, [AlignedSegment]) of a BAM file."""
    raw = gzip.decompress(open(path, "rb").read())
    assert raw[:4] == b"BAM\x01"
    o = 4
    lt = struct.unpack_from("<i", raw, o)[0]
    o += 4 + lt
    nref = struct.unpack_from("<i", raw, o)[0]
    o += 4
    refs = []
    for _ in range(nref):
        ln = struct.unpack_from("<i", raw, o)[0]
        name = raw[o + 4:o + 4 + ln - 1].decode()
        o += 4 + ln
        refs.append((name, struct.unpack_from("<i", raw, o)[0]))
        o += 4
    recs = []
    while o < len(raw):
        bs = struct.unpack_from("<i", raw, o)[0]
        ref, pos, lrn, _mq, _bin, ncig, flag, lseq = struct.unpack_from("<iiBBHHHi", raw, o + 4)
        p = o + 36
        name = raw[p:p + lrn - 1].decode()
        p += lrn
        cig = [(v & 15, v >> 4) for v in struct.unpack_from("<%dI" % ncig, raw, p)]
        p += 4 * ncig
        sb = raw[p:p + (lseq + 1) // 2]
        seq = "".join(SEQ_CODES[(sb[i // 2] >> (4 * (1 - i % 2))) & 15] for i in range(lseq)) if lseq else None
        recs.append(AlignedSegment(refs, ref, pos, flag, name, cig, seq))
        o += 4 + bs
    return refs, recs


class AlignmentFile:
    """pysam.AlignmentFile stand-in for reading ("rb")."""

    def __init__(self, path, mode="rb"):
        self._refs, self._recs = read_bam(path)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __iter__(self):
        return iter(self._recs)
