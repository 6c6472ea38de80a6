"""The C++ host API (include/tfusion/topfu.hpp, the tfusion::TopFu mirror) and the headless
demo that replays apps/demo.cpp's loop over it."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APPS = os.path.join(ROOT, "apps")


def _build():
    subprocess.run(["make", "-s", "-C", APPS], check=True)
    return os.path.join(APPS, "demo_headless")


def test_cpp_api_builds_and_links():
    exe = _build()
    assert os.path.exists(exe)
    syms = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for fn in ("tf_create", "tf_process_frame", "tf_render_image", "tf_destroy"):
        assert fn in syms


@pytest.mark.gpu
def test_demo_headless_runs():
    exe = _build()
    r = subprocess.run([exe, "40", "320", "240"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"frames (\d+) ok (\d+) resets (\d+)", r.stdout)
    assert m and int(m.group(1)) == 40 and int(m.group(2)) >= 30, r.stdout
    assert "rendered pixels lit" in r.stdout
