"""Frame files: the reference demo's %04d.pgm / %04d.ppm pairs
(apps/demo.cpp:91-97), read by topfusion_amd.io and by include/tfusion/io.hpp."""
import os
import subprocess

import numpy as np

from topfusion_amd import io, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pgm_ppm_round_trip(tmp_path):
    d = synth.orbit_sequence(1, 64, 48)[0]
    d[0, 0], d[1, 1] = 65535, 0x1234            # byte order matters
    io.write_pgm16(tmp_path / "0000.pgm", d)
    assert np.array_equal(io.read_pgm16(tmp_path / "0000.pgm"), d)
    raw = open(tmp_path / "0000.pgm", "rb").read()
    assert raw.endswith(d.astype(">u2").tobytes())  # big-endian samples, as netpbm specifies
    bgr = np.random.default_rng(1).integers(0, 256, (48, 64, 3), dtype=np.uint8)
    io.write_ppm(tmp_path / "0000.ppm", bgr)
    assert np.array_equal(io.read_ppm(tmp_path / "0000.ppm"), bgr)


def test_pgm_header_comments_and_8bit(tmp_path):
    p = tmp_path / "c.pgm"
    pix = np.arange(12, dtype=np.uint8).reshape(3, 4)
    open(p, "wb").write(b"P5\n# a comment\n4 3\n# another\n255\n" + pix.tobytes())
    assert np.array_equal(io.read_pgm16(p), pix.astype(np.uint16))


def test_cpp_reader_matches(tmp_path):
    """include/tfusion/io.hpp reads the same pixels (FrameSequenceSource over a %04d pattern)."""
    seq = synth.orbit_sequence(3, 40, 30)
    for i, f in enumerate(seq):
        io.write_pgm16(tmp_path / f"{i:04d}.pgm", f)
        io.write_ppm(tmp_path / f"{i:04d}.ppm", np.stack([f & 255, f >> 8, f * 0 + i], -1).astype(np.uint8))
    src = tmp_path / "rd.cpp"
    src.write_text(r'''
#include <tfusion/io.hpp>
#include <cstdio>
int main(int, char** argv) {
    tfusion::io::FrameSequenceSource s(std::string(argv[1]) + "/%04d.pgm", std::string(argv[1]) + "/%04d.ppm");
    std::vector<uint16_t> d; std::vector<uint8_t> c;
    while (s.grab(d, c)) {
        unsigned long long h = 1469598103934665603ull;
        for (uint16_t v : d) h = (h ^ v) * 1099511628211ull;
        for (uint8_t v : c) h = (h ^ v) * 1099511628211ull;
        std::printf("%d %d %llu\n", s.cols(), s.rows(), h);
    }
    return 0;
}''')
    exe = tmp_path / "rd"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, check=True).stdout.split("\n")
    assert len([l for l in out if l]) == 3
    for i in range(3):
        d = io.read_pgm16(tmp_path / f"{i:04d}.pgm")
        c = io.read_ppm(tmp_path / f"{i:04d}.ppm")
        h = 1469598103934665603
        for v in d.reshape(-1).tolist():
            h = ((h ^ v) * 1099511628211) & (2 ** 64 - 1)
        for v in c.reshape(-1).tolist():
            h = ((h ^ v) * 1099511628211) & (2 ** 64 - 1)
        assert out[i] == f"40 30 {h}", (out[i], h)
