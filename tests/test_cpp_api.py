"""The C++ host API (include/tfusion/topfu.hpp, the tfusion::TopFu mirror) and the headless
demo that replays apps/demo.cpp's loop over it."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APPS = os.path.join(ROOT, "apps")


def _build(app="demo_headless"):
    subprocess.run(["make", "-s", "-C", APPS], check=True)
    return os.path.join(APPS, app)


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
    # SampledScopeTime's function-static counter (core.cpp:206-216): one scope per frame prints
    # the average once, at the 34th
    assert r.stdout.count("Average frame time = ") == 1, r.stdout


def test_engine_api_builds_and_links():
    exe = _build("engine_check")
    syms = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for fn in ("tf_scene_alloc", "tf_scene_integrate", "tf_vis_render_image", "tf_vis_icp_maps", "tf_icp_estimate",
               "tf_imgproc_bilateral", "tf_icp_set_params"):
        assert fn in syms, fn


def test_swap_api_builds_and_links():
    exe = _build("swap_check")
    syms = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for fn in ("tf_scene_swap_in", "tf_scene_swap_out", "tf_swap_save", "tf_swap_load", "tf_download_range"):
        assert fn in syms, fn


@pytest.mark.gpu
def test_swap_api_runs(tmp_path):
    """apps/swap_check: a swapping Scene over the engine API (SwappingEngine_CUDA's two calls
    after allocation + integration), free-list bookkeeping every frame, GlobalCache
    SaveToFile / ReadFromFile into a second scene."""
    exe = _build("swap_check")
    r = subprocess.run([exe, str(tmp_path / "cache.bin")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"swapped in (\d+) out (\d+) stored (\d+): MATCH", r.stdout)
    assert m and int(m.group(2)) > 0 and int(m.group(3)) > 0, r.stdout


def test_colour_api_builds_and_links():
    exe = _build("colour_check")
    syms = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for fn in ("tf_process_frame_rgb", "tf_scene_integrate_rgb", "tf_render_image_type", "tf_vis_render_image"):
        assert fn in syms, fn


@pytest.mark.gpu
def test_colour_api_matches_topfu():
    """apps/colour_check: TopFu::operator()(depth, rgba) with integrate_colour against the same
    frames over a Scene<Voxel_s_rgb> and IntegrateIntoScene(..., rgb): hash, voxel plane, colour
    plane and RENDER_COLOUR_FROM_VOLUME bit-exact; an unregistered colour camera."""
    exe = _build("colour_check")
    r = subprocess.run([exe, "24", "320", "240"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"coloured voxels (\d+) lit pixels (\d+): MATCH", r.stdout)
    assert m and int(m.group(1)) > 10000 and int(m.group(2)) > 10000, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("wait", ["wait", "nowait"])
def test_engine_api_matches_topfu(wait):
    """apps/engine_check: TopFu::operator() against the same frames spelled out over the L4
    engine API (imgproc functions, a stand-alone ProjectiveICP, the reconstruction and
    visualisation engines) -- bool, pose, counters and renderImage bit-exact every frame, ICP
    maps at the end; 40 frames include ICP-failure resets.  "nowait" leaves out the
    cuda::waitAllDefaultStream() between the imgproc calls (asynchronous, legacy default
    stream) and the engines: AllocateSceneFromDepth right after computeDists, estimateTransform
    right after computePointNormals -- the entry points order themselves after stream 0."""
    exe = _build("engine_check")
    r = subprocess.run([exe, "40", "320", "240", wait], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"engine_check frames (\d+) ok (\d+) resets (\d+): MATCH", r.stdout)
    assert m and int(m.group(1)) == 40 and int(m.group(3)) >= 1, r.stdout


@pytest.mark.gpu
def test_demo_headless_pgm_sequence(tmp_path):
    """The demo over a %04d.pgm / %04d.ppm sequence (the reference demo's input format,
    apps/demo.cpp:91-97), read through tfusion::io::FrameSequenceSource."""
    import numpy as np
    from topfusion_amd import io, synth
    seq = synth.orbit_sequence(12, 320, 240, seed=7)
    for i, f in enumerate(seq):
        io.write_pgm16(tmp_path / f"{i:04d}.pgm", f)
        io.write_ppm(tmp_path / f"{i:04d}.ppm", np.zeros((240, 320, 3), np.uint8))
    exe = _build()
    r = subprocess.run([exe, "--pgm", str(tmp_path / "%04d.pgm"), "--ppm", str(tmp_path / "%04d.ppm")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"frames (\d+) ok (\d+) resets (\d+)", r.stdout)
    assert m and int(m.group(1)) == 12 and int(m.group(2)) >= 8, r.stdout


def test_cv_types_alias_compiles():
    """where OpenCV exists the tfusion value types are OpenCV's own
    (include/tfusion/types.hpp, TFUSION_OPENCV_TYPES), so apps/demo.cpp's uses -- TopFu::Ptr as
    cv::Ptr (demo.cpp:30), params.volume_size / volume_pose and getCameraPose() handed to cv::viz
    (:34-35, :115), cuda::DeviceArray<Point> (:146), OpenNISource (io/capture.hpp) -- compile with
    no conversion.  Compile-only, against the stand-in cv headers of tests/cvstub (OpenCV is absent
    from this image)."""
    src = os.path.join(ROOT, "tests", "cvstub", "demo_api_check.cpp")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-DTFUSION_OPENCV_TYPES=1",
                        "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "tests", "cvstub"),
                        "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # and without OpenCV (this image) the same headers pick their own types
    probe = ('#include <tfusion/types.hpp>\n#include <type_traits>\n'
             'static_assert(TFUSION_OPENCV_TYPES == 0, "no OpenCV here");\n'
             'static_assert(std::is_same<tfusion::SharedPtr<int>, std::shared_ptr<int>>::value, "");\nint main(){}\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-x", "c++", "-D__HIP_PLATFORM_AMD__",
                        "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", "-"],
                       input=probe, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


REF_DEMO = "/root/reference/apps/demo.cpp"


@pytest.mark.skipif(not os.path.exists(REF_DEMO), reason="the reference tree is not on this machine")
def test_reference_demo_compiles():
    """the reference's own apps/demo.cpp -- the file itself, read where it lies,
    not an extract -- compiles against include/ (tfusion/topfu.hpp, tfusion/types.hpp,
    io/capture.hpp) with TFUSION_OPENCV_TYPES on.  Compile-only (-fsyntax-only), against the
    stand-in OpenCV headers of tests/cvstub (core, highgui, imgproc, viz: the declarations demo.cpp
    uses, with OpenCV's public signatures; OpenCV is absent from this image)."""
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-DTFUSION_OPENCV_TYPES=1", "-D__HIP_PLATFORM_AMD__",
                        "-I", os.path.join(ROOT, "tests", "cvstub"), "-I", os.path.join(ROOT, "include"),
                        "-I", "/opt/rocm/include", REF_DEMO],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
