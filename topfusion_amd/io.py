"""Frame files of the reference demo (apps/demo.cpp:91-97): 16-bit PGM depth + 8-bit PPM colour.

Same pixels as OpenCV's imread(path, CV_16U) / imread(path) for binary netpbm files: P5 with
maxval > 255 holds big-endian 16-bit samples; P6 holds RGB, returned as BGR like imread.
The C++ side is include/tfusion/io.hpp (readPGM16 / readPPM / FrameSequenceSource)."""
import numpy as np


def _header(buf, magic):
    if buf[:2] != magic:
        raise ValueError(f"not a binary {magic.decode()} file")
    fields, i = [], 2
    while len(fields) < 3:
        while buf[i:i + 1] in (b" ", b"\t", b"\r", b"\n") or buf[i:i + 1] == b"#":
            if buf[i:i + 1] == b"#":
                while buf[i:i + 1] not in (b"\n", b""):
                    i += 1
            i += 1
        j = i
        while buf[j:j + 1].isdigit():
            j += 1
        if j == i:
            raise ValueError("bad netpbm header")
        fields.append(int(buf[i:j]))
        i = j
    return fields, i + 1            # one whitespace byte ends the header


def read_pgm16(path):
    """(rows, cols) uint16 depth of a P5 PGM."""
    buf = open(path, "rb").read()
    (cols, rows, maxval), off = _header(buf, b"P5")
    if maxval > 255:
        return np.frombuffer(buf, ">u2", cols * rows, off).reshape(rows, cols).astype(np.uint16)
    return np.frombuffer(buf, np.uint8, cols * rows, off).reshape(rows, cols).astype(np.uint16)


def write_pgm16(path, depth):
    d = np.ascontiguousarray(depth, np.uint16)
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n65535\n" % (d.shape[1], d.shape[0]))
        f.write(d.astype(">u2").tobytes())


def read_ppm(path):
    """(rows, cols, 3) uint8 B, G, R of a P6 PPM."""
    buf = open(path, "rb").read()
    (cols, rows, maxval), off = _header(buf, b"P6")
    if maxval > 255:
        raise ValueError("16-bit PPM not supported")
    rgb = np.frombuffer(buf, np.uint8, cols * rows * 3, off).reshape(rows, cols, 3)
    return rgb[..., ::-1].copy()


def write_ppm(path, bgr):
    b = np.ascontiguousarray(bgr, np.uint8)
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (b.shape[1], b.shape[0]))
        f.write(b[..., ::-1].tobytes())


def read_sequence(depth_pattern, first=0, count=None):
    """Frames depth_pattern % i for i = first, first+1, ... until the first missing file."""
    import os
    out, i = [], first
    while (count is None or len(out) < count) and os.path.exists(depth_pattern % i):
        out.append(read_pgm16(depth_pattern % i))
        i += 1
    return np.stack(out) if out else np.zeros((0, 0, 0), np.uint16)
