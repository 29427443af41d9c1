"""RDEIC bitstream container (utils/utils.py:30-80): big-endian uint32 header (z_h, z_w,
n_strings = 2), then for each string a big-endian uint32 length and the bytes; the y (rANS)
string comes first, the z (hyper-latent, torchac) string second (compression.py:211)."""
from __future__ import annotations

import struct
from pathlib import Path
from typing import List, Sequence, Tuple


def pack_body(shape: Sequence[int], strings: Sequence[Sequence[bytes]]) -> bytes:
    out = [struct.pack(">3I", int(shape[0]), int(shape[1]), len(strings))]
    for s in strings:
        out.append(struct.pack(">I", len(s[0])))
        out.append(bytes(s[0]))
    return b"".join(out)


def unpack_body(data: bytes) -> Tuple[List[List[bytes]], Tuple[int, int]]:
    """Inverse of pack_body. Truncated input raises struct.error / ValueError like the reference."""
    if len(data) < 12:
        raise struct.error("unpack requires a buffer of 12 bytes")
    zh, zw, n = struct.unpack_from(">3I", data, 0)
    pos = 12
    strings = []
    for _ in range(n):
        (ln,) = struct.unpack_from(">I", data, pos)
        pos += 4
        if pos + ln > len(data):
            raise ValueError("truncated bitstream")
        strings.append([bytes(data[pos:pos + ln])])
        pos += ln
    return strings, (zh, zw)


def write_body(fd, shape, out_strings) -> int:
    body = pack_body(shape, out_strings)
    fd.write(body)
    return len(body)


def read_body(fd):
    return unpack_body(fd.read())


def filesize(filepath: str) -> int:
    p = Path(filepath)
    if not p.is_file():
        raise ValueError(f'Invalid file "{filepath}".')
    return p.stat().st_size
