"""Python mirror of the reference's pipeline API (tfusion/include/tfusion/topfu.hpp:28-110)
over the C-ABI of libtfusion_hip.so.

    params = TopFuParams.default_params()     # topfu.cpp:12-53
    topfu = TopFu(params)                     # topfu.cpp:55-84
    ok = topfu(depth)                         # operator(), topfu.cpp:161-330
    img = topfu.renderImage()                 # topfu.cpp:332-377
    pose = topfu.getCameraPose()              # topfu.cpp:154-159
    topfu.reset()                             # topfu.cpp:141-152

`depth` is a uint16 (rows, cols) numpy array (host; uploaded like cuda::Depth::upload)
or a device pointer (int) to uint16 millimetres on the context's device.
"""
import ctypes

import numpy as np

from . import _lib as L

HASH_DTYPE = np.dtype([("x", "<i2"), ("y", "<i2"), ("z", "<i2"), ("pad", "<i2"), ("offset", "<i4"), ("ptr", "<i4")])
VOXEL_DTYPE = np.dtype([("sdf", "<i2"), ("w", "u1"), ("pad", "u1")])


class TopFuParams:
    """TopFuParams: construct with default_params() and override attributes."""

    @staticmethod
    def default_params(**kw):
        return L.default_params(**kw)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _rt(m):
    a = np.ascontiguousarray(np.asarray(m, np.float32)[:3, :4] if np.ndim(m) == 2 else np.asarray(m, np.float32))
    return a.reshape(12)


class TopFu:
    """tfusion::TopFu on one MI355X (one HIP stream per instance)."""

    def __init__(self, params=None, device=None, **kw):
        lib = L.load()
        if device is not None:
            L.check(lib.tf_set_device(int(device)), "tf_set_device")
        self.params_ = params if params is not None else L.default_params(**kw)
        h = ctypes.c_void_p()
        L.check(lib.tf_create(ctypes.byref(self.params_), ctypes.byref(h)), "tf_create")
        self._h = h
        self.W, self.H = self.params_.cols, self.params_.rows
        self.n_total = self.params_.n_buckets + self.params_.n_excess
        self._framed = False

    def close(self):
        if getattr(self, "_h", None):
            L.load().tf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def params(self):
        return self.params_

    # -- TopFu API ----------------------------------------------------------------------
    def __call__(self, depth, pitch=0, rgb=None):
        """TopFu::operator()(depth, image): returns the frame's bool (False = ICP failed, scene
        reset).  rgb (voxel_rgb contexts): the frame's uchar4 (rows, cols, 4) image -- a host array
        with a host depth, a device pointer with a device depth."""
        lib = L.load()
        pose = np.zeros(12, np.float32)
        if isinstance(depth, int):
            if rgb is None:
                s = lib.tf_process_frame(self._h, ctypes.c_void_p(depth), pitch, _ptr(pose), None)
            else:
                s = lib.tf_process_frame_rgb(self._h, ctypes.c_void_p(depth), pitch, ctypes.c_void_p(int(rgb)), 0,
                                             _ptr(pose), None)
        else:
            d = np.ascontiguousarray(depth, np.uint16)
            assert d.shape == (self.H, self.W), d.shape
            if rgb is None:
                s = lib.tf_process_frame_host(self._h, _ptr(d), self.W * 2, _ptr(pose), None)
            else:
                c = np.ascontiguousarray(rgb, np.uint8)
                assert c.shape == (self.H, self.W, 4), c.shape
                s = lib.tf_process_frame_rgb_host(self._h, _ptr(d), self.W * 2, _ptr(c), self.W * 4, _ptr(pose),
                                                  None)
        L.check(s, "tf_process_frame", allow=(L.TF_OK, L.TF_ICP_FAIL))
        self._framed = True
        return s == L.TF_OK

    def process_frames(self, dev_frames, n, stride=None, rgb_frames=None, rgb_stride=None):
        """Runs n device-resident frames (and, voxel_rgb, their device-resident RGB images);
        returns the per-frame bools."""
        ok = np.zeros(n, np.int32)
        stride = stride if stride is not None else self.W * self.H * 2
        if rgb_frames is None:
            L.check(L.load().tf_process_frames(self._h, ctypes.c_void_p(dev_frames), stride, n, _ptr(ok)),
                    "tf_process_frames")
        else:
            rs = rgb_stride if rgb_stride is not None else self.W * self.H * 4
            L.check(L.load().tf_process_frames_rgb(self._h, ctypes.c_void_p(dev_frames), stride,
                                                   ctypes.c_void_p(int(rgb_frames)), rs, n, _ptr(ok)),
                    "tf_process_frames_rgb")
        return ok.astype(bool)

    def renderImage(self, type=0):
        """TopFu::renderImage -> uint8 (rows, cols, 4) image (host copy).  type: the reference's
        IVisualisationEngine::RenderImageType (0 shaded greyscale = TopFu::renderImage, 1 greyscale
        from image normals, 2 colour from volume (greyscale for Voxel_s), 3 colour from normal,
        4 colour from confidence)."""
        L.check(L.load().tf_render_image_type(self._h, int(type), None, 0), "tf_render_image_type")
        return self.download(L.TF_BUF_GREY).view(np.uint8).reshape(self.H, self.W, 4)

    def frame_grey(self):
        """The grey image renderImage produced inside the last tracked frame (no re-render)."""
        return self.download(L.TF_BUF_GREY).view(np.uint8).reshape(self.H, self.W, 4)

    def getCameraPose(self):
        rt = np.zeros(12, np.float32)
        L.check(L.load().tf_get_pose(self._h, _ptr(rt)), "tf_get_pose")
        m = np.eye(4, dtype=np.float32)
        m[:3, :4] = rt.reshape(3, 4)
        return m

    def reset(self):
        L.check(L.load().tf_reset(self._h), "tf_reset")

    @property
    def last_stats(self):
        """The counters after the last frame (tf_get_stats: waits for the frame's remaining work --
        a frame call returns once its result is known, with its later stages still running)."""
        return self.stats() if self._framed else None

    def stats(self):
        s = L.TfStats()
        L.check(L.load().tf_get_stats(self._h, ctypes.byref(s)), "tf_get_stats")
        return s.as_dict()

    def totals(self):
        """Frame totals accumulated on the device since creation / reset_totals() (tf_totals)."""
        t = L.TfTotals()
        L.check(L.load().tf_get_totals(self._h, ctypes.byref(t)), "tf_get_totals")
        return t.as_dict()

    def reset_totals(self):
        L.check(L.load().tf_reset_totals(self._h), "tf_reset_totals")

    def stream(self):
        return L.load().tf_get_stream(self._h)

    POSE_ALGEBRAS = {"canonical": 0, "opencv2": 2, "opencv4": 4, "svd": 4}

    def set_pose_algebra(self, algebra):
        """The ICP iterations' det / solve / Rodrigues (tf_set_pose_algebra): the reference's OpenCV
        algebra, "opencv4" (default; = "svd") or "opencv2" (2.4.9), or "canonical" (LU + 2 x 2 block
        Schur solve + sinc Rodrigues: a shorter serial tail, not the reference's arithmetic)."""
        a = self.POSE_ALGEBRAS[algebra] if isinstance(algebra, str) else int(algebra)
        L.check(L.load().tf_set_pose_algebra(self._h, a), "tf_set_pose_algebra")

    def pose_algebra(self):
        v = ctypes.c_int()
        L.check(L.load().tf_get_pose_algebra(self._h, ctypes.byref(v)), "tf_get_pose_algebra")
        return v.value

    def icp_persistent(self):
        """True when ICP runs as one persistent launch per frame."""
        v = ctypes.c_int()
        L.check(L.load().tf_get_schedule(self._h, ctypes.byref(v)), "tf_get_schedule")
        return bool(v.value)

    # -- per-stage HIP-event timing ----------------------------------------------------
    def profile(self, enable=True, stages=None, every=1):
        """Time every stage (enable=True), none, or only the named stages (HIP events on the
        context stream; each timed stage costs GPU time of its own), on every `every`-th frame."""
        if stages is None:
            L.check(L.load().tf_profile_enable(self._h, int(enable)), "tf_profile_enable")
        else:
            mask = 0
            for s in stages:
                mask |= 1 << L.STAGE_NAMES.index(s)
            L.check(L.load().tf_profile_stages(self._h, mask if enable else 0), "tf_profile_stages")
        L.check(L.load().tf_profile_sample(self._h, int(every)), "tf_profile_sample")
        L.check(L.load().tf_profile_reset(self._h), "tf_profile_reset")

    def profile_read(self):
        n = len(L.STAGE_NAMES)
        ms = np.zeros(n, np.float64)
        cnt = np.zeros(n, np.int64)
        L.check(L.load().tf_profile_read(self._h, _ptr(ms), _ptr(cnt), n), "tf_profile_read")
        return {name: (float(ms[i]), int(cnt[i])) for i, name in enumerate(L.STAGE_NAMES)}

    # -- stage entry points (parity tests) ------------------------------------------------
    def stage_preprocess(self, depth):
        """computeDists + bilateral + truncation + pyramid + vertex/normal maps (host depth)."""
        d = np.ascontiguousarray(depth, np.uint16)
        assert d.shape == (self.H, self.W), d.shape
        L.check(L.load().tf_stage_preprocess_host(self._h, _ptr(d), self.W * 2), "tf_stage_preprocess_host")

    def stage_icp(self):
        aff = np.zeros(12, np.float32)
        ok = ctypes.c_int()
        it = ctypes.c_int()
        L.check(L.load().tf_stage_icp(self._h, _ptr(aff), ctypes.byref(ok), ctypes.byref(it)), "tf_stage_icp")
        return bool(ok.value), aff.reshape(3, 4), it.value

    def stage_alloc(self, pose_rt):
        L.check(L.load().tf_stage_alloc(self._h, _ptr(_rt(pose_rt))), "tf_stage_alloc")

    def stage_integrate(self, pose_rt):
        L.check(L.load().tf_stage_integrate(self._h, _ptr(_rt(pose_rt))), "tf_stage_integrate")

    def stage_expected_depths(self, pose_rt):
        L.check(L.load().tf_stage_expected_depths(self._h, _ptr(_rt(pose_rt))), "tf_stage_expected_depths")

    def stage_raycast(self, invM_rt, update_visible):
        L.check(L.load().tf_stage_raycast(self._h, _ptr(_rt(invM_rt)), int(update_visible)), "tf_stage_raycast")

    def stage_icp_maps(self, invM_rt):
        L.check(L.load().tf_stage_icp_maps(self._h, _ptr(_rt(invM_rt))), "tf_stage_icp_maps")

    def stage_render_grey(self, invM_rt):
        L.check(L.load().tf_stage_render_grey(self._h, _ptr(_rt(invM_rt))), "tf_stage_render_grey")
        return self.download(L.TF_BUF_GREY).view(np.uint8).reshape(self.H, self.W, 4)

    def stage_reset_scene(self):
        L.check(L.load().tf_stage_reset_scene(self._h), "tf_stage_reset_scene")

    def stage_swap_pyramids(self):
        L.check(L.load().tf_stage_swap_pyramids(self._h), "tf_stage_swap_pyramids")

    # -- state transfer ------------------------------------------------------------------
    def nbytes(self, which, level=0):
        n = ctypes.c_size_t()
        L.check(L.load().tf_buffer_bytes(self._h, which, level, ctypes.byref(n)), "tf_buffer_bytes")
        return n.value

    def download(self, which, level=0):
        n = self.nbytes(which, level)
        buf = np.empty(n, np.uint8)
        L.check(L.load().tf_download(self._h, which, level, _ptr(buf), n), "tf_download")
        return buf

    def upload(self, which, arr, level=0):
        a = np.ascontiguousarray(arr)
        n = self.nbytes(which, level)
        assert a.nbytes == n, (a.nbytes, n)
        L.check(L.load().tf_upload(self._h, which, level, _ptr(a), n), "tf_upload")

    def set_pose(self, rt):
        L.check(L.load().tf_set_pose(self._h, _ptr(_rt(rt))), "tf_set_pose")

    def time_stage(self, stage, pose_rt, iters):
        """ms per launch of `iters` back-to-back launches of a stage's kernels (HIP events on
        the context stream); stage: "integrate" or "raycast_icp"."""
        ms = ctypes.c_float()
        L.check(L.load().tf_time_stage(self._h, L.STAGE_NAMES.index(stage), _ptr(_rt(pose_rt)), int(iters),
                                       ctypes.byref(ms)), "tf_time_stage")
        return float(ms.value)

    def set_counters(self, lastFreeBlockId, lastFreeExcessListId, noVisibleEntries):
        L.check(L.load().tf_set_counters(self._h, lastFreeBlockId, lastFreeExcessListId, noVisibleEntries),
                "tf_set_counters")

    def fuse_frames(self, dev_frames, poses_w2c, stride=None, pitch=0, intr=None):
        """tf_scene_fuse_frames: computeDists + AllocateSceneFromDepth + IntegrateIntoScene (+ the
        swapping engine) per frame of a device-resident uint16 batch (`dev_frames`: device address
        of frame 0) at the world->camera poses `poses_w2c` (n x 3 x 4 or n x 12); returns the
        per-frame records (numpy structured array, L.FUSE_RECORD_DTYPE)."""
        P = np.ascontiguousarray(np.asarray(poses_w2c, np.float32).reshape(-1, 12))
        n = len(P)
        rec = np.zeros(n, L.FUSE_RECORD_DTYPE)
        if stride is None:
            stride = self.W * self.H * 2
        ip = None if intr is None else _ptr(np.ascontiguousarray(intr, np.float32))
        L.check(L.load().tf_scene_fuse_frames(self._h, ip, ctypes.c_void_p(int(dev_frames)), int(stride), int(pitch),
                                              _ptr(P), n, _ptr(rec)), "tf_scene_fuse_frames")
        return rec

    def alloc_list(self):
        """LocalVBA::allocationList (the free-block stack)."""
        return self.download(L.TF_BUF_ALLOC_LIST).view(np.int32)

    def excess_list(self):
        return self.download(L.TF_BUF_EXCESS_LIST).view(np.int32)

    # swapping (GlobalCache in HBM)
    def swap(self):
        """The swapping engine once (IntegrateGlobalIntoLocal + SaveToGlobalMemory)."""
        L.check(L.load().tf_scene_swap(self._h), "tf_scene_swap")

    def swap_in(self):
        """IntegrateGlobalIntoLocal alone."""
        L.check(L.load().tf_scene_swap_in(self._h), "tf_scene_swap_in")

    def swap_out(self):
        """SaveToGlobalMemory alone."""
        L.check(L.load().tf_scene_swap_out(self._h), "tf_scene_swap_out")

    def swap_counts(self):
        """(swapped in, swapped out, reallocated) blocks of the last frame / call."""
        out = np.zeros(3, np.int32)
        L.check(L.load().tf_swap_counts(self._h, _ptr(out)), "tf_swap_counts")
        return tuple(int(v) for v in out)

    def swap_state(self):
        return self.download(L.TF_BUF_SWAP_STATE)

    def swap_stored_flags(self):
        return self.download(L.TF_BUF_SWAP_STORED_FLAGS)

    def swap_stored(self):
        return self.download(L.TF_BUF_SWAP_STORED).view(VOXEL_DTYPE)

    def swap_save(self, path):
        L.check(L.load().tf_swap_save(self._h, str(path).encode()), "tf_swap_save")

    def swap_load(self, path):
        L.check(L.load().tf_swap_load(self._h, str(path).encode()), "tf_swap_load")

    # typed views
    def hash(self):
        return self.download(L.TF_BUF_HASH).view(HASH_DTYPE)

    def vba(self):
        return self.download(L.TF_BUF_VBA).view(VOXEL_DTYPE)

    def vba_rgb(self):
        """voxel_rgb: the colour plane, uint32 per voxel (r | g << 8 | b << 16 | w_color << 24)."""
        return self.download(L.TF_BUF_VBA_RGB).view(np.uint32)

    def visible_ids(self):
        n = self.stats()["noVisibleEntries"]
        return self.download(L.TF_BUF_VISIBLE_IDS).view(np.int32)[:n]

    def visible_type(self):
        return self.download(L.TF_BUF_VISIBLE_TYPE)

    def range_image(self):
        return self.download(L.TF_BUF_RANGE).view(np.float32).reshape(self.H, self.W, 2)

    def raycast_result(self):
        return self.download(L.TF_BUF_RAYCAST).view(np.float32).reshape(self.H, self.W, 4)

    def dists(self):
        return self.download(L.TF_BUF_DISTS).view(np.float32).reshape(self.H, self.W)

    def level_shape(self, l):
        return self.H >> l, self.W >> l

    def curr_depth(self, l):
        return self.download(L.TF_BUF_DEPTH, l).view(np.uint16).reshape(self.level_shape(l))

    def curr_maps(self, l):
        h, w = self.level_shape(l)
        return (self.download(L.TF_BUF_CURR_POINTS, l).view(np.float32).reshape(h, w, 4),
                self.download(L.TF_BUF_CURR_NORMALS, l).view(np.float32).reshape(h, w, 4))

    def prev_maps(self, l):
        h, w = self.level_shape(l)
        return (self.download(L.TF_BUF_PREV_POINTS, l).view(np.float32).reshape(h, w, 4),
                self.download(L.TF_BUF_PREV_NORMALS, l).view(np.float32).reshape(h, w, 4))
