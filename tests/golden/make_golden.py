"""Regenerates the reference-pinned golden vectors in tests/golden/ (run in the build
container, where /root/reference exists; the GPU box only reads the committed files).

  1. `make -C oracle ref` compiles oracle/ref_pin/ref_pin.cpp against the reference's own,
     self-contained headers (tfusion/include/Math.hpp, Vector.hpp, Matrix.hpp,
     MathUtils.hpp, tfusion/cuda/VoxelTypes.hpp, tfusion/cuda/PixelUtils.hpp) into
     oracle/_ref/ref_pin -- no stand-in
     headers, nothing from the reference is copied into the repo.
  2. oracle/_ref/ref_pin writes ref_pin_{inv,m4v,round,voxel,bilinear,colour}.bin here (raw little-endian
     f32 records; layouts in tests/test_oracle.py).

    python tests/golden/make_golden.py
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def main():
    if not os.path.isdir("/root/reference/tfusion/include"):
        sys.exit("reference tree absent: the committed goldens stay as they are")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_pin"), HERE], check=True)


if __name__ == "__main__":
    main()
