"""ctypes binding of libtfusion_hip.so (the C-ABI declared in include/tfusion_hip.h).

The shared library is built in-tree by topfusion_amd/csrc/Makefile (hipcc, gfx950).
There is no CPU fallback: if the library is missing, loading fails loudly.
"""
import ctypes
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TFUSION_HIP_LIB") or os.path.join(_HERE, "libtfusion_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "tfusion_hip.h")

TF_OK, TF_ICP_FAIL, TF_INVALID_ARG, TF_OOM, TF_HIP_ERROR, TF_NO_DEVICE = range(6)

STAGE_NAMES = ("preprocess", "icp", "alloc", "integrate", "raycast_render", "grey", "expected_depths",
               "raycast_icp", "icp_maps")

(TF_BUF_HASH, TF_BUF_VBA, TF_BUF_VISIBLE_IDS, TF_BUF_VISIBLE_TYPE, TF_BUF_RANGE, TF_BUF_RAYCAST, TF_BUF_DISTS,
 TF_BUF_DEPTH, TF_BUF_CURR_POINTS, TF_BUF_CURR_NORMALS, TF_BUF_PREV_POINTS, TF_BUF_PREV_NORMALS, TF_BUF_GREY,
 TF_BUF_SWAP_STATE, TF_BUF_SWAP_STORED_FLAGS, TF_BUF_SWAP_STORED, TF_BUF_VBA_RGB, TF_BUF_ALLOC_LIST,
 TF_BUF_EXCESS_LIST) = range(19)


class TfParams(ctypes.Structure):
    """tf_params (include/tfusion_hip.h) == TopFuParams + SceneParams + capacities."""
    _fields_ = [("cols", ctypes.c_int), ("rows", ctypes.c_int),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("bilateral_sigma_depth", ctypes.c_float), ("bilateral_sigma_spatial", ctypes.c_float),
                ("bilateral_kernel_size", ctypes.c_int),
                ("icp_truncate_depth_dist", ctypes.c_float), ("icp_dist_thres", ctypes.c_float),
                ("icp_angle_thres", ctypes.c_float), ("icp_iter_num", ctypes.c_int * 4),
                ("mu", ctypes.c_float), ("maxW", ctypes.c_int), ("voxelSize", ctypes.c_float),
                ("viewFrustum_min", ctypes.c_float), ("viewFrustum_max", ctypes.c_float),
                ("n_buckets", ctypes.c_int), ("n_excess", ctypes.c_int), ("n_blocks", ctypes.c_int),
                ("vis_capacity", ctypes.c_int), ("max_render_blocks", ctypes.c_int),
                ("use_swapping", ctypes.c_int), ("swap_transfer_blocks", ctypes.c_int),
                ("voxel_rgb", ctypes.c_int), ("rgb_intr", ctypes.c_float * 4), ("depth_to_rgb", ctypes.c_float * 12)]


class TfStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("lastFreeBlockId", "lastFreeExcessListId", "noVisibleEntries",
                                            "noTotalBlocks", "frame_counter", "icp_iterations", "icp_ok",
                                            "n_resets")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class TfTotals(ctypes.Structure):
    _fields_ = [(n, ctypes.c_longlong) for n in ("frames", "frames_tracked", "resets", "visible_sum", "tiles_sum",
                                                 "swapped_in", "swapped_out", "integrate_lanes_read",
                                                 "integrate_lanes_written", "swapped_in_merged",
                                                 "alloc_failed_type1", "alloc_failed_type2", "icp_fallbacks")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


FUSE_RECORD_FIELDS = ("lastFreeBlockId", "lastFreeExcessListId", "noVisibleEntries", "alloc_failed_type1",
                      "alloc_failed_type2", "swapped_in", "swapped_out", "swap_realloc", "swapped_in_merged", "pad")
FUSE_RECORD_DTYPE = np.dtype([(n, "<i4") for n in FUSE_RECORD_FIELDS])   # tf_fuse_record


class TfMapLevel(ctypes.Structure):
    """tf_map_level: one level of a float4 point / normal pyramid (device pointers, row steps)."""
    _fields_ = [("points", ctypes.c_void_p), ("points_step", ctypes.c_size_t),
                ("normals", ctypes.c_void_p), ("normals_step", ctypes.c_size_t)]


class TfError(RuntimeError):
    def __init__(self, status, where):
        self.status = status
        super().__init__(f"{where}: tf_status {status} ({status_string(status)})")


_lib = None


def header_functions():
    """Names of every function declared in include/tfusion_hip.h."""
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tf_[a-z0-9_]+)\s*\(", src)))


def load():
    """Load libtfusion_hip.so (no fallback: raises if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `make -C topfusion_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    S = ctypes.c_size_t
    sig = {
        "tf_device_count": ([ctypes.POINTER(I)], I),
        "tf_set_device": ([I], I),
        "tf_status_string": ([I], ctypes.c_char_p),
        "tf_default_params": ([ctypes.POINTER(TfParams)], I),
        "tf_create": ([ctypes.POINTER(TfParams), ctypes.POINTER(P)], I),
        "tf_destroy": ([P], None),
        "tf_reset": ([P], I),
        "tf_process_frame": ([P, P, S, P, ctypes.POINTER(TfStats)], I),
        "tf_process_frame_host": ([P, P, S, P, ctypes.POINTER(TfStats)], I),
        "tf_process_frames": ([P, P, S, I, P], I),
        "tf_process_frame_rgb": ([P, P, S, P, S, P, ctypes.POINTER(TfStats)], I),
        "tf_process_frame_rgb_host": ([P, P, S, P, S, P, ctypes.POINTER(TfStats)], I),
        "tf_process_frames_rgb": ([P, P, S, P, S, I, P], I),
        "tf_render_image": ([P, P, S], I),
        "tf_get_pose": ([P, P], I),
        "tf_get_stats": ([P, ctypes.POINTER(TfStats)], I),
        "tf_get_params": ([P, ctypes.POINTER(TfParams)], I),
        "tf_get_stream": ([P], P),
        "tf_get_schedule": ([P, ctypes.POINTER(I)], I),
        "tf_set_pose_algebra": ([P, I], I),
        "tf_get_pose_algebra": ([P, ctypes.POINTER(I)], I),
        "tf_icp_solve_systems": ([I, P, I, P, P, P], I),
        "tf_stage_preprocess": ([P, P, S], I),
        "tf_stage_preprocess_host": ([P, P, S], I),
        "tf_stage_icp": ([P, P, ctypes.POINTER(I), ctypes.POINTER(I)], I),
        "tf_stage_alloc": ([P, P], I),
        "tf_stage_integrate": ([P, P], I),
        "tf_stage_expected_depths": ([P, P], I),
        "tf_stage_raycast": ([P, P, I], I),
        "tf_stage_icp_maps": ([P, P], I),
        "tf_stage_render_grey": ([P, P], I),
        "tf_stage_reset_scene": ([P], I),
        "tf_stage_swap_pyramids": ([P], I),
        "tf_buffer_bytes": ([P, I, I, ctypes.POINTER(S)], I),
        "tf_download": ([P, I, I, P, S], I),
        "tf_download_range": ([P, I, S, P, S], I),
        "tf_upload": ([P, I, I, P, S], I),
        "tf_set_pose": ([P, P], I),
        "tf_set_counters": ([P, I, I, I], I),
        "tf_get_totals": ([P, ctypes.POINTER(TfTotals)], I),
        "tf_icp_set_params": ([P, F, F, P], I),
        "tf_icp_get_params": ([P, ctypes.POINTER(F), ctypes.POINTER(F), P], I),
        "tf_icp_estimate": ([P, P, ctypes.POINTER(TfMapLevel), ctypes.POINTER(TfMapLevel), I, P,
                             ctypes.POINTER(I), ctypes.POINTER(I)], I),
        "tf_scene_alloc": ([P, P, P, P, S, I, I], I),
        "tf_scene_integrate": ([P, P, P, P, S], I),
        "tf_scene_integrate_rgb": ([P, P, P, P, S, P, S], I),
        "tf_vis_expected_depths": ([P, P, P], I),
        "tf_scene_swap": ([P], I),
        "tf_scene_fuse_frames": ([P, P, P, S, S, P, I, P], I),
        "tf_scene_swap_in": ([P], I),
        "tf_scene_swap_out": ([P], I),
        "tf_swap_counts": ([P, P], I),
        "tf_swap_save": ([P, ctypes.c_char_p], I),
        "tf_swap_load": ([P, ctypes.c_char_p], I),
        "tf_vis_render_image": ([P, P, P, I, I, P, S], I),
        "tf_vis_icp_maps": ([P, P, P, P, S, P, S], I),
        "tf_imgproc_compute_dists": ([P, S, P, S, I, I, P], I),
        "tf_imgproc_bilateral": ([P, S, P, S, I, I, I, F, F, P], I),
        "tf_imgproc_truncate": ([P, S, I, I, F, P], I),
        "tf_imgproc_pyr_down": ([P, S, I, I, P, S, F, P], I),
        "tf_imgproc_point_normals": ([P, P, S, I, I, P, S, P, S, P], I),
        "tf_imgproc_resize_points_normals": ([P, S, P, S, I, I, P, S, P, S, P], I),
        "tf_imgproc_sync": ([P], I),
        "tf_reset_totals": ([P], I),
        "tf_render_image_type": ([P, I, P, S], I),
        "tf_time_stage": ([P, I, P, I, ctypes.POINTER(ctypes.c_float)], I),
        "tf_profile_enable": ([P, I], I),
        "tf_profile_stages": ([P, ctypes.c_uint], I),
        "tf_profile_sample": ([P, I], I),
        "tf_profile_reset": ([P], I),
        "tf_profile_read": ([P, P, P, I], I),
    }
    override = bool(os.environ.get("TFUSION_HIP_LIB"))    # an A/B build (tools/gpu_ab_c3i.sh) may be older
    for name, (args, res) in sig.items():
        if override and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def status_string(s):
    try:
        return load().tf_status_string(int(s)).decode()
    except Exception:
        return str(s)


def check(status, where, allow=(TF_OK,)):
    if status not in allow:
        raise TfError(status, where)
    return status


def device_count():
    """HIP devices visible to this process (tf_device_count)."""
    n = ctypes.c_int(0)
    check(load().tf_device_count(ctypes.byref(n)), "tf_device_count")
    return n.value


def default_params(**kw):
    p = TfParams()
    check(load().tf_default_params(ctypes.byref(p)), "tf_default_params")
    for k, v in kw.items():
        if k == "icp_iter_num":
            for i in range(4):
                p.icp_iter_num[i] = int(v[i]) if i < len(v) else 0
        elif k in ("rgb_intr", "depth_to_rgb"):
            arr = getattr(p, k)
            for i, x in enumerate(v):
                arr[i] = float(x)
        else:
            setattr(p, k, v)
    return p
