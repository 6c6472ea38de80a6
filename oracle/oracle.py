"""ctypes wrapper around the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product (topfusion_amd/).
See oracle/tf_oracle.h for what is pinned and what is "parity unpinned".
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_LIB_OMP = os.path.join(_HERE, "liboracle_omp.so")      # same source, OpenMP loops enabled


class Params(ctypes.Structure):
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


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("lastFreeBlockId", "lastFreeExcessListId", "noVisibleEntries",
                                            "noTotalBlocks", "frame_counter", "icp_iterations", "icp_ok",
                                            "n_resets")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


HASH_DTYPE = np.dtype([("x", "<i2"), ("y", "<i2"), ("z", "<i2"), ("pad", "<i2"), ("offset", "<i4"), ("ptr", "<i4")])
VOXEL_DTYPE = np.dtype([("sdf", "<i2"), ("w", "u1"), ("pad", "u1")])

_libs = {}


def build(omp=False):
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle_omp.so" if omp else "liboracle.so"], check=True)


def lib(omp=False):
    """The serial oracle (default) or its OpenMP build (omp=True: the all-cores CPU baseline;
    every result identical, tests/test_oracle.py)."""
    if omp not in _libs:
        path = _LIB_OMP if omp else _LIB
        build(omp)                  # make: a no-op unless the sources are newer
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.tfo_default_params.argtypes = [ctypes.POINTER(Params)]
        L.tfo_exp.argtypes = [ctypes.c_float]; L.tfo_exp.restype = ctypes.c_float
        L.tfo_interp_bilinear_u8x4.argtypes = [P, ctypes.c_size_t, ctypes.c_float, ctypes.c_float, P]
        L.tfo_colour_average.argtypes = [ctypes.c_uint32, P, ctypes.c_int]; L.tfo_colour_average.restype = ctypes.c_uint32
        L.tfo_compute_dists.argtypes = [P, ctypes.c_int, ctypes.c_int, P]
        L.tfo_bilateral.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float]
        L.tfo_truncate.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_float]
        L.tfo_pyr_down.argtypes = [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_float]
        L.tfo_points_normals.argtypes = [P, ctypes.c_int, ctypes.c_int] + [ctypes.c_float] * 4 + [P, P]
        L.tfo_resize_points_normals.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, P]
        L.tfo_icp_reduce.argtypes = [P, P, P, P, ctypes.c_int, ctypes.c_int] + [ctypes.c_float] * 6 + [P, P]
        L.tfo_icp_step.argtypes = [P, P, ctypes.POINTER(ctypes.c_double)]; L.tfo_icp_step.restype = ctypes.c_int
        L.tfo_rigid_mul.argtypes = [P, P, P]
        L.tfo_rigid_inv.argtypes = [P, P]
        L.tfo_matrix4_inv.argtypes = [P, P]; L.tfo_matrix4_inv.restype = ctypes.c_int
        L.tfo_m4v.argtypes = [P, P, P]
        L.tfo_tsdf_update.argtypes = [P, P, ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.tfo_sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.tfo_rodrigues.argtypes = [P, P]
        L.tfo_rodrigues_direct.argtypes = [P, P]
        L.tfo_set_pose_algebra.argtypes = [ctypes.c_int, ctypes.c_int]
        L.tfo_get_pose_algebra.restype = ctypes.c_int
        L.tfo_cv_det6.argtypes = [P, ctypes.c_int]; L.tfo_cv_det6.restype = ctypes.c_double
        L.tfo_cv_jacobi_svd.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int]
        L.tfo_cv_solve_svd6.argtypes = [P, P, P]
        L.tfo_solve6.argtypes = [P, P, P]
        L.tfo_det6.argtypes = [P]; L.tfo_det6.restype = ctypes.c_double
        L.tfo_cv_rodrigues.argtypes = [P, P, ctypes.c_int]
        L.tfo_cv_svd_stats.argtypes = [P, ctypes.c_int]
        L.tfo_capture_sums.argtypes = [P, ctypes.c_longlong]
        L.tfo_captured_sums.restype = ctypes.c_longlong
        L.tfo_cv_hypot.argtypes = [ctypes.c_double, ctypes.c_double]; L.tfo_cv_hypot.restype = ctypes.c_double
        L.tfo_point_conv.argtypes = [P, P]
        L.tfo_hash_index.argtypes = [ctypes.c_int] * 4; L.tfo_hash_index.restype = ctypes.c_int
        L.tfo_create.argtypes = [ctypes.POINTER(Params)]; L.tfo_create.restype = P
        L.tfo_destroy.argtypes = [P]
        L.tfo_reset.argtypes = [P]
        L.tfo_reset_scene.argtypes = [P]
        L.tfo_swap_merged_total.argtypes = [P]; L.tfo_swap_merged_total.restype = ctypes.c_longlong
        L.tfo_copy_state.argtypes = [P, P]; L.tfo_copy_state.restype = ctypes.c_int
        L.tfo_process_frame.argtypes = [P, P]; L.tfo_process_frame.restype = ctypes.c_int
        L.tfo_get_counters.argtypes = [P, ctypes.POINTER(Counters)]
        L.tfo_set_counters.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.tfo_get_pose.argtypes = [P, P]
        L.tfo_alloc.argtypes = [P, P, P]
        L.tfo_alloc_ex.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int]
        L.tfo_integrate.argtypes = [P, P, P]
        L.tfo_integrate_rgb.argtypes = [P, P, P, P, ctypes.c_size_t]
        L.tfo_process_frame_rgb.argtypes = [P, P, P, ctypes.c_size_t]; L.tfo_process_frame_rgb.restype = ctypes.c_int
        L.tfo_expected_depths.argtypes = [P, P]
        L.tfo_raycast.argtypes = [P, P, ctypes.c_int]
        L.tfo_render_icp.argtypes = [P, P, P, P]
        L.tfo_render_grey.argtypes = [P, P, P]
        L.tfo_render_image.argtypes = [P, P]
        L.tfo_render_type.argtypes = [P, P, ctypes.c_int, P]
        L.tfo_render_image_type.argtypes = [P, ctypes.c_int]
        L.tfo_swap.argtypes = [P]
        L.tfo_swap_in.argtypes = [P]
        L.tfo_swap_out.argtypes = [P]
        L.tfo_swap_counts.argtypes = [P, P]
        L.tfo_alloc_failures.argtypes = [P, P]
        for name in ("tfo_alloc_list", "tfo_excess_list", "tfo_hash", "tfo_vba", "tfo_visible_ids", "tfo_visible_type", "tfo_range_image",
                     "tfo_raycast_result", "tfo_dists", "tfo_frame_grey", "tfo_swap_state", "tfo_swap_stored_flags",
                     "tfo_swap_stored", "tfo_vba_rgb"):
            getattr(L, name).argtypes = [P]; getattr(L, name).restype = P
        for name in ("tfo_prev_points", "tfo_prev_normals", "tfo_curr_points", "tfo_curr_normals", "tfo_curr_depth"):
            getattr(L, name).argtypes = [P, ctypes.c_int]; getattr(L, name).restype = P
        _libs[omp] = L
    return _libs[omp]


POSE_CANONICAL, POSE_OPENCV2, POSE_OPENCV4 = 0, 2, 4
POSE_MODES = {"canonical": POSE_CANONICAL, "opencv2": POSE_OPENCV2, "opencv4": POSE_OPENCV4}


def set_pose_algebra(mode, libm=False, omp=None):
    """Test-only: the pose algebra estimateTransform's iterations use (tf_oracle.c, "The
    reference's own pose algebra"): "opencv4" (the default, as the GPU's) / "opencv2"
    (cv::determinant, cv::solve DECOMP_SVD and Affine3f(rvec, t) as OpenCV 3.x-4.x / 2.4.9 publish
    them, restated: not checked against an OpenCV build) or "canonical" (LU + block Schur + sinc
    Rodrigues), with glibc's (libm=True) or the portable sin / cos / hypot.
    Applies to the serial and (omp=None) the OpenMP build alike."""
    m = POSE_MODES[mode] if isinstance(mode, str) else int(mode)
    for o in ((False, True) if omp is None else (omp,)):
        lib(o).tfo_set_pose_algebra(m, 1 if libm else 0)


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def default_params(**kw):
    p = Params()
    lib().tfo_default_params(ctypes.byref(p))
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


# ---- stateless stages -------------------------------------------------------

def compute_dists(depth):
    H, W = depth.shape
    out = np.empty((H, W), np.float32)
    lib().tfo_compute_dists(ptr(np.ascontiguousarray(depth, np.uint16)), W, H, ptr(out))
    return out


def bilateral(depth, ksz=7, sigma_spatial=4.5, sigma_depth=0.04):
    H, W = depth.shape
    src = np.ascontiguousarray(depth, np.uint16)
    out = np.empty_like(src)
    lib().tfo_bilateral(ptr(src), ptr(out), W, H, ksz, sigma_spatial, sigma_depth)
    return out


def truncate(depth, max_dist=2.0):
    H, W = depth.shape
    out = np.ascontiguousarray(depth, np.uint16).copy()
    lib().tfo_truncate(ptr(out), W, H, max_dist)
    return out


def pyr_down(depth, sigma_depth=0.04):
    H, W = depth.shape
    src = np.ascontiguousarray(depth, np.uint16)
    out = np.empty((H // 2, W // 2), np.uint16)
    lib().tfo_pyr_down(ptr(src), W, H, ptr(out), sigma_depth)
    return out


def points_normals(depth, fx, fy, cx, cy):
    H, W = depth.shape
    src = np.ascontiguousarray(depth, np.uint16)
    pts = np.empty((H, W, 4), np.float32)
    nrm = np.empty((H, W, 4), np.float32)
    lib().tfo_points_normals(ptr(src), W, H, fx, fy, cx, cy, ptr(pts), ptr(nrm))
    return pts, nrm


def resize_points_normals(pts, nrm):
    H, W = pts.shape[:2]
    po = np.empty((H // 2, W // 2, 4), np.float32)
    no = np.empty((H // 2, W // 2, 4), np.float32)
    lib().tfo_resize_points_normals(ptr(np.ascontiguousarray(pts)), ptr(np.ascontiguousarray(nrm)), W, H, ptr(po), ptr(no))
    return po, no


def icp_reduce(vcurr, ncurr, vprev, nprev, fx, fy, cx, cy, min_cosine, dist2_thres, aff):
    H, W = vcurr.shape[:2]
    out = np.empty(27, np.float32)
    a = np.ascontiguousarray(aff, np.float32).reshape(12)
    lib().tfo_icp_reduce(ptr(vcurr), ptr(ncurr), ptr(vprev), ptr(nprev), W, H, fx, fy, cx, cy,
                         min_cosine, dist2_thres, ptr(a), ptr(out))
    return out


def icp_step(sums27, affine):
    a = np.ascontiguousarray(affine, np.float32).reshape(12).copy()
    s = np.ascontiguousarray(sums27, np.float32)
    det = ctypes.c_double()
    ok = lib().tfo_icp_step(ptr(s), ptr(a), ctypes.byref(det))
    return bool(ok), a, det.value


def matrix4_inv(m):
    m = np.ascontiguousarray(m, np.float32).reshape(16)
    out = np.zeros(16, np.float32)
    ok = lib().tfo_matrix4_inv(ptr(m), ptr(out))
    return bool(ok), out


def m4v(m, v):
    out = np.zeros(4, np.float32)
    lib().tfo_m4v(ptr(np.ascontiguousarray(m, np.float32)), ptr(np.ascontiguousarray(v, np.float32)), ptr(out))
    return out


def tsdf_update(sdf, w, eta, mu=0.02, maxW=100):
    s = np.array([sdf], np.int16)
    ww = np.array([w], np.uint8)
    lib().tfo_tsdf_update(ptr(s), ptr(ww), eta, mu, maxW)
    return int(s[0]), int(ww[0])


def interp_bilinear_u8x4(rgba, x, y):
    """interpolateBilinear<uchar> (PixelUtils.hpp:8-32) of an HxWx4 uint8 image at (x, y)."""
    img = np.ascontiguousarray(rgba, np.uint8)
    out = np.zeros(4, np.float32)
    lib().tfo_interp_bilinear_u8x4(ptr(img), img.shape[1] * 4, x, y, ptr(out))
    return out


def colour_average(rgb, w, sample, maxW=100):
    """computeUpdatedVoxelColorInfo's running average (SceneReconstructionEngine.hpp:124-147):
    (r, g, b), w_color and an interpolated sample -> (r', g', b'), w_color'."""
    clr = int(rgb[0]) | (int(rgb[1]) << 8) | (int(rgb[2]) << 16) | (int(w) << 24)
    s = np.zeros(4, np.float32)
    s[:3] = sample[:3]
    o = lib().tfo_colour_average(clr, ptr(s), maxW)
    return (o & 255, (o >> 8) & 255, (o >> 16) & 255), o >> 24


# ---- stateful pipeline -------------------------------------------------------

class Oracle:
    """The reference TopFu pipeline restated on the CPU (oracle/tf_oracle.c)."""

    def __init__(self, params=None, omp=False, **kw):
        self.L = lib(omp)
        self.params = params if params is not None else default_params(**kw)
        self.ctx = self.L.tfo_create(ctypes.byref(self.params))
        self.W, self.H = self.params.cols, self.params.rows
        self.n_total = self.params.n_buckets + self.params.n_excess

    def __del__(self):
        try:
            if getattr(self, "ctx", None):
                self.L.tfo_destroy(self.ctx)
                self.ctx = None
        except Exception:
            pass

    def __call__(self, depth, rgb=None):
        d = np.ascontiguousarray(depth, np.uint16)
        assert d.shape == (self.H, self.W)
        if rgb is None:
            return bool(self.L.tfo_process_frame(self.ctx, ptr(d)))
        c = np.ascontiguousarray(rgb, np.uint8)
        assert c.shape == (self.H, self.W, 4)
        return bool(self.L.tfo_process_frame_rgb(self.ctx, ptr(d), ptr(c), 0))

    def reset(self):
        self.L.tfo_reset(self.ctx)

    def swap_merged_total(self):
        """Swap-ins that merged stored data (GlobalCache -> VBA transfers) since creation."""
        return int(self.L.tfo_swap_merged_total(self.ctx))

    def reset_scene(self):
        """SceneReconstructionEngine::ResetScene (the GlobalCache stays)."""
        self.L.tfo_reset_scene(self.ctx)

    def copy_state_from(self, other):
        """This context's whole state := other's (same params; either build may be the source)."""
        assert self.L.tfo_copy_state(self.ctx, other.ctx) == 0, "tfo_copy_state: params differ"

    def counters(self):
        c = Counters()
        self.L.tfo_get_counters(self.ctx, ctypes.byref(c))
        return c.as_dict()

    def pose(self):
        rt = np.zeros(12, np.float32)
        self.L.tfo_get_pose(self.ctx, ptr(rt))
        return rt.reshape(3, 4)

    def _view(self, addr, dtype, count, shape=None):
        buf = (ctypes.c_char * (np.dtype(dtype).itemsize * count)).from_address(addr)
        a = np.frombuffer(buf, dtype=dtype, count=count)
        return a.reshape(shape) if shape else a

    def hash(self):
        return self._view(self.L.tfo_hash(self.ctx), HASH_DTYPE, self.n_total).copy()

    def upload_hash(self, h):
        """Write a whole hash table (HASH_DTYPE, n_total entries) into the context."""
        h = np.ascontiguousarray(h, HASH_DTYPE)
        assert h.shape == (self.n_total,)
        self._view(self.L.tfo_hash(self.ctx), HASH_DTYPE, self.n_total)[:] = h

    def alloc_list(self):
        """LocalVBA::allocationList, the free-block stack."""
        return self._view(self.L.tfo_alloc_list(self.ctx), np.int32, self.params.n_blocks).copy()

    def excess_list(self):
        return self._view(self.L.tfo_excess_list(self.ctx), np.int32, self.params.n_excess).copy()

    def alloc_failures(self):
        """(type-1, type-2) allocation requests the last AllocateSceneFromDepth refused."""
        out = np.zeros(2, np.int32)
        self.L.tfo_alloc_failures(self.ctx, ptr(out))
        return int(out[0]), int(out[1])

    def load_scene_state(self, hash, vba, alloc_list, excess_list, visible_ids, visible_type, counters,
                         swap_state=None, swap_stored_flags=None, swap_stored=None):
        """Overwrite the scene and render-state arrays the engine-level passes read (a state taken
        from another implementation, e.g. the GPU's at frame k of a stream): hash, voxels, both
        free lists, the visible list and types, the counters (lastFreeBlockId,
        lastFreeExcessListId, noVisibleEntries) and, in a swapping scene, the GlobalCache."""
        n_tot, nb = self.n_total, self.params.n_blocks
        self._view(self.L.tfo_hash(self.ctx), HASH_DTYPE, n_tot)[:] = np.asarray(hash, HASH_DTYPE)
        self._view(self.L.tfo_vba(self.ctx), VOXEL_DTYPE, nb * 512)[:] = np.asarray(vba, VOXEL_DTYPE)
        self._view(self.L.tfo_alloc_list(self.ctx), np.int32, nb)[:] = alloc_list
        self._view(self.L.tfo_excess_list(self.ctx), np.int32, self.params.n_excess)[:] = excess_list
        self._view(self.L.tfo_visible_ids(self.ctx), np.int32, self.params.vis_capacity)[:] = visible_ids
        self._view(self.L.tfo_visible_type(self.ctx), np.uint8, n_tot)[:] = visible_type
        self.set_counters(*counters)
        if self.params.use_swapping:
            self._view(self.L.tfo_swap_state(self.ctx), np.uint8, n_tot)[:] = swap_state
            self._view(self.L.tfo_swap_stored_flags(self.ctx), np.uint8, n_tot)[:] = swap_stored_flags
            self._view(self.L.tfo_swap_stored(self.ctx), VOXEL_DTYPE, n_tot * 512)[:] = np.asarray(swap_stored, VOXEL_DTYPE)

    def upload_visible_ids(self, ids):
        ids = np.ascontiguousarray(ids, np.int32)
        assert ids.size <= self.params.vis_capacity
        self._view(self.L.tfo_visible_ids(self.ctx), np.int32, self.params.vis_capacity)[:ids.size] = ids

    def set_counters(self, lastFreeBlockId, lastFreeExcessListId, noVisibleEntries):
        self.L.tfo_set_counters(self.ctx, lastFreeBlockId, lastFreeExcessListId, noVisibleEntries)

    def vba(self):
        return self._view(self.L.tfo_vba(self.ctx), VOXEL_DTYPE, self.params.n_blocks * 512).copy()

    def vba_rgb(self):
        """voxel_rgb: the colour plane, uint32 per voxel (r | g << 8 | b << 16 | w_color << 24)."""
        return self._view(self.L.tfo_vba_rgb(self.ctx), np.uint32, self.params.n_blocks * 512).copy()

    def visible_ids(self):
        n = self.counters()["noVisibleEntries"]
        return self._view(self.L.tfo_visible_ids(self.ctx), np.int32, self.params.vis_capacity)[:n].copy()

    def visible_type(self):
        return self._view(self.L.tfo_visible_type(self.ctx), np.uint8, self.n_total).copy()

    def range_image(self):
        return self._view(self.L.tfo_range_image(self.ctx), np.float32, self.W * self.H * 2, (self.H, self.W, 2)).copy()

    def raycast_result(self):
        return self._view(self.L.tfo_raycast_result(self.ctx), np.float32, self.W * self.H * 4, (self.H, self.W, 4)).copy()

    def frame_grey(self):
        return self._view(self.L.tfo_frame_grey(self.ctx), np.uint8, self.W * self.H * 4, (self.H, self.W, 4)).copy()

    def dists(self):
        return self._view(self.L.tfo_dists(self.ctx), np.float32, self.W * self.H, (self.H, self.W)).copy()

    def level_shape(self, l):
        return self.H >> l, self.W >> l

    def prev_maps(self, l):
        h, w = self.level_shape(l)
        p = self._view(self.L.tfo_prev_points(self.ctx, l), np.float32, h * w * 4, (h, w, 4)).copy()
        n = self._view(self.L.tfo_prev_normals(self.ctx, l), np.float32, h * w * 4, (h, w, 4)).copy()
        return p, n

    def curr_maps(self, l):
        h, w = self.level_shape(l)
        p = self._view(self.L.tfo_curr_points(self.ctx, l), np.float32, h * w * 4, (h, w, 4)).copy()
        n = self._view(self.L.tfo_curr_normals(self.ctx, l), np.float32, h * w * 4, (h, w, 4)).copy()
        return p, n

    def curr_depth(self, l):
        h, w = self.level_shape(l)
        return self._view(self.L.tfo_curr_depth(self.ctx, l), np.uint16, h * w, (h, w)).copy()

    # stage-level
    def alloc(self, pose_rt, dists, only_update_visible=False, reset_visible=False):
        self.L.tfo_alloc_ex(self.ctx, ptr(np.ascontiguousarray(pose_rt, np.float32).reshape(12)),
                            ptr(np.ascontiguousarray(dists, np.float32)), int(only_update_visible), int(reset_visible))

    def integrate(self, pose_rt, dists, rgb=None):
        pr = ptr(np.ascontiguousarray(pose_rt, np.float32).reshape(12))
        dd = np.ascontiguousarray(dists, np.float32)
        if rgb is None:
            self.L.tfo_integrate(self.ctx, pr, ptr(dd))
        else:
            c = np.ascontiguousarray(rgb, np.uint8)
            assert c.shape == (self.H, self.W, 4)
            self.L.tfo_integrate_rgb(self.ctx, pr, ptr(dd), ptr(c), 0)

    def expected_depths(self, pose_rt):
        self.L.tfo_expected_depths(self.ctx, ptr(np.ascontiguousarray(pose_rt, np.float32).reshape(12)))

    def raycast(self, invM_rt, update_visible):
        self.L.tfo_raycast(self.ctx, ptr(np.ascontiguousarray(invM_rt, np.float32).reshape(12)), int(update_visible))

    def render_icp(self, invM_rt):
        pts = np.empty((self.H, self.W, 4), np.float32)
        nrm = np.empty((self.H, self.W, 4), np.float32)
        self.L.tfo_render_icp(self.ctx, ptr(np.ascontiguousarray(invM_rt, np.float32).reshape(12)), ptr(pts), ptr(nrm))
        return pts, nrm

    def render_grey(self, invM_rt):
        img = np.empty((self.H, self.W, 4), np.uint8)
        self.L.tfo_render_grey(self.ctx, ptr(np.ascontiguousarray(invM_rt, np.float32).reshape(12)), ptr(img))
        return img

    def render_image(self):
        img = np.empty((self.H, self.W, 4), np.uint8)
        self.L.tfo_render_image(self.ctx, ptr(img))
        return img

    # swapping state (GlobalCache)
    def swap(self):
        """The swapping engine once (IntegrateGlobalIntoLocal + SaveToGlobalMemory)."""
        self.L.tfo_swap(self.ctx)

    def swap_in(self):
        self.L.tfo_swap_in(self.ctx)

    def swap_out(self):
        self.L.tfo_swap_out(self.ctx)

    def swap_counts(self):
        """Last frame's (swapped in, swapped out, reallocated) block counts."""
        out = np.zeros(3, np.int32)
        self.L.tfo_swap_counts(self.ctx, ptr(out))
        return tuple(int(v) for v in out)

    def swap_state(self):
        return self._view(self.L.tfo_swap_state(self.ctx), np.uint8, self.n_total).copy()

    def swap_stored_flags(self):
        return self._view(self.L.tfo_swap_stored_flags(self.ctx), np.uint8, self.n_total).copy()

    def swap_stored(self):
        return self._view(self.L.tfo_swap_stored(self.ctx), VOXEL_DTYPE, self.n_total * 512).copy()

    def render_image_type(self, type):
        """RenderImage(type) from the current pose into the context image (the buffer the frame's
        renderImage fills, so alpha-preserving types see its previous content); returns a copy."""
        self.L.tfo_render_image_type(self.ctx, int(type))
        return self.frame_grey()


def point_conv(p):
    out = np.zeros(13, np.float32)
    lib().tfo_point_conv(ptr(np.ascontiguousarray(p, np.float32)), ptr(out))
    return out


def sincos(th):
    s, c = ctypes.c_double(), ctypes.c_double()
    lib().tfo_sincos(float(th), ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


def rodrigues(r):
    R = np.zeros(9, np.float32)
    lib().tfo_rodrigues(ptr(np.ascontiguousarray(r, np.float32)), ptr(R))
    return R.reshape(3, 3)


def rigid_mul(a, b):
    out = np.zeros(12, np.float32)
    lib().tfo_rigid_mul(ptr(np.ascontiguousarray(a, np.float32).reshape(12)),
                        ptr(np.ascontiguousarray(b, np.float32).reshape(12)), ptr(out))
    return out.reshape(3, 4)


def rigid_inv(a):
    out = np.zeros(12, np.float32)
    lib().tfo_rigid_inv(ptr(np.ascontiguousarray(a, np.float32).reshape(12)), ptr(out))
    return out.reshape(3, 4)


def hash_index(x, y, z, n_buckets=0x100000):
    return int(lib().tfo_hash_index(int(x), int(y), int(z), int(n_buckets)))
