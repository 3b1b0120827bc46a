"""Test helpers: a small PNG encoder (every row filter type, colour types 0/2/4/6) and a reference
decoder in numpy, used to check the library's PNG front end (fd_png_*)."""
import struct
import zlib

import numpy as np


def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def encode_png(img, filters=(0, 1, 2, 3, 4)):
    """img: uint8 [rows, cols] (gray) or [rows, cols, C] with C in 2/3/4; row r uses filters[r % len]."""
    img = np.ascontiguousarray(img, np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    rows, cols, ch = img.shape
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[ch]
    stride = cols * ch
    raw = bytearray()
    prev = np.zeros(stride, np.int32)
    for r in range(rows):
        cur = img[r].reshape(-1).astype(np.int32)
        ft = filters[r % len(filters)]
        a = np.concatenate([np.zeros(ch, np.int32), cur[:-ch]])
        c = np.concatenate([np.zeros(ch, np.int32), prev[:-ch]])
        pred = {0: np.zeros_like(cur), 1: a, 2: prev, 3: (a + prev) >> 1, 4: _paeth(a, prev, c)}[ft]
        raw.append(ft)
        raw += ((cur - pred) & 0xFF).astype(np.uint8).tobytes()
        prev = cur
    hdr = struct.pack(">IIBBBBB", cols, rows, 8, ctype, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", hdr) + _chunk(b"IDAT", zlib.compress(bytes(raw))) + _chunk(b"IEND", b"")


def decode_png(data):
    """Reference decoder (numpy): samples [rows, cols, C]."""
    pos, idat = 8, b""
    while pos < len(data):
        n = int.from_bytes(data[pos:pos + 4], "big")
        t, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if t == b"IHDR":
            cols, rows = int.from_bytes(body[0:4], "big"), int.from_bytes(body[4:8], "big")
            ch = {0: 1, 4: 2, 2: 3, 6: 4}[body[9]]
        elif t == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8)
    stride = cols * ch
    out = np.zeros((rows, stride), np.int32)
    prev = [0] * stride
    for r in range(rows):
        ft = int(raw[r * (stride + 1)])
        line = raw[r * (stride + 1) + 1:(r + 1) * (stride + 1)].tolist()
        if ft in (0, 2):
            cur = [(v + (0 if ft == 0 else p)) & 0xFF for v, p in zip(line, prev)]
        else:
            cur = [0] * stride
            for i in range(stride):
                a = cur[i - ch] if i >= ch else 0
                b = prev[i]
                c = prev[i - ch] if i >= ch else 0
                if ft == 1:
                    p = a
                elif ft == 3:
                    p = (a + b) >> 1
                else:
                    pp = a + b - c
                    pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
                    p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                cur[i] = (line[i] + p) & 0xFF
        out[r] = cur
        prev = cur
    return out.astype(np.uint8).reshape(rows, cols, ch)


def gray_of(samples):
    """The library's colour -> gray: (4899 R + 9617 G + 1868 B + 8192) >> 14; alpha dropped."""
    s = samples.astype(np.uint32)
    if s.shape[2] <= 2:
        return s[:, :, 0].astype(np.uint8)
    return ((4899 * s[:, :, 0] + 9617 * s[:, :, 1] + 1868 * s[:, :, 2] + 8192) >> 14).astype(np.uint8)
