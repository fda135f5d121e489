"""ORBextractor mirror (include/ORBextractor.h:35-81) over the gfx950 C-ABI."""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import KP_DTYPE, OrbxParams, check, lib, ptr, stream_ptr, tptr


@dataclass
class Parameters:
    """ORBextractor::Parameters (include/ORBextractor.h:39-47; defaults src/ORBextractor.cc:830-833)."""
    nfeatures: int = 2000
    scaleFactor: float = 1.2
    nlevels: int = 8
    iniThFAST: int = 20
    minThFAST: int = 7

    def c(self):
        return OrbxParams(self.nfeatures, self.scaleFactor, self.nlevels, self.iniThFAST, self.minThFAST)


class ORBextractor:
    Parameters = Parameters

    def __init__(self, param: Parameters = None, device: int = 0):
        self.param = param or Parameters()
        self._h = C.c_void_p()
        check(lib().orbx_create(C.byref(self.param.c()), device, C.byref(self._h)), "orbx_create")
        L = self.param.nlevels
        self._scale, self._inv, self._s2, self._is2 = (np.zeros(L, np.float32) for _ in range(4))
        self._quota = np.zeros(L, np.int32)
        check(lib().orbx_scale_tables(self._h, ptr(self._scale), ptr(self._inv), ptr(self._s2), ptr(self._is2),
                                      ptr(self._quota)), "orbx_scale_tables")
        self._last_shape = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().orbx_destroy(h)
            except Exception:
                pass
            self._h = None

    # -- getters (src/ORBextractor.cc:822-828)
    def GetLevels(self):
        return self.param.nlevels

    def GetScaleFactor(self):
        return self.param.scaleFactor

    def GetScaleFactors(self):
        return self._scale.copy()

    def GetInverseScaleFactors(self):
        return self._inv.copy()

    def GetScaleSigmaSquares(self):
        return self._s2.copy()

    def GetInverseScaleSigmaSquares(self):
        return self._is2.copy()

    def FeaturesPerLevel(self):
        return self._quota.copy()

    TRIG_MODES = {"double": 0, "float": 1}

    def set_opencv_compat(self, trig=None, resize_simd=None):
        """The OpenCV-build switches (include/orbslam2_amd.h orbx_set_opencv_compat): trig "double"
        (::cos(double), default) or "float" (cosf / sinf) for ComputeOrbDescriptor's cos / sin
        (src/ORBextractor.cc:107); resize_simd = the build's SIMD width V in bytes for cv::resize's
        scalar tail (0 default = SIMD rounding everywhere, as OpenCV's uchar VResizeLinear; 8-64 = a
        FixedPtCast tail after a V-byte loop, 1 = FixedPtCast everywhere: sensitivity switches).  None keeps."""
        t = -1 if trig is None else self.TRIG_MODES[trig] if isinstance(trig, str) else int(trig)
        v = -1 if resize_simd is None else int(resize_simd)
        check(lib().orbx_set_opencv_compat(self._h, t, v), "orbx_set_opencv_compat")

    def get_opencv_compat(self):
        t, v = C.c_int(0), C.c_int(0)
        check(lib().orbx_get_opencv_compat(self._h, C.byref(t), C.byref(v)), "orbx_get_opencv_compat")
        return ("double", "float")[t.value], v.value

    def max_keypoints(self, rows, cols):
        cap = C.c_int32(0)
        check(lib().orbx_max_keypoints(self._h, rows, cols, C.byref(cap)), "orbx_max_keypoints")
        return cap.value

    def Extract(self, image: np.ndarray, keypoints=None):
        """void Extract(const cv::Mat& image, KeyPoints& keypoints, cv::Mat& descriptors).

        Returns (keypoints, descriptors).  Reference quirk (src/ORBextractor.cc:778-782): when the
        image yields no keypoint the descriptors are released (None) and the caller's `keypoints`
        argument is returned unchanged.
        """
        img = np.asarray(image)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("image must be CV_8U single channel")   # CV_Assert (:457)
        if img.strides[1] != 1:
            img = np.ascontiguousarray(img)
        rows, cols = img.shape
        cap = self.max_keypoints(rows, cols)
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        check(lib().orbx_extract(self._h, ptr(img), rows, cols, C.c_size_t(img.strides[0]), ptr(kps), ptr(desc), cap,
                                 C.byref(n)), "orbx_extract")
        self._last_shape = (rows, cols)
        if n.value == 0:
            return keypoints, None
        return kps[:n.value].copy(), desc[:n.value].copy()

    __call__ = Extract

    def GetImagePyramid(self):
        """Levels of the last extracted image (unblurred), as numpy arrays."""
        out = []
        for l in range(self.param.nlevels):
            r, c = C.c_int(0), C.c_int(0)
            check(lib().orbx_pyramid_level(self._h, l, None, 0, C.byref(r), C.byref(c)), "orbx_pyramid_level")
            a = np.zeros((r.value, c.value), np.uint8)
            check(lib().orbx_pyramid_level(self._h, l, ptr(a), c.value, C.byref(r), C.byref(c)), "orbx_pyramid_level")
            out.append(a)
        return out

    STAGES = ("pyramid", "fast_cells", "quadtree", "describe")

    def profile(self, enable: bool = True, stages=None):
        """Per-kernel event timing of every stage, or only of `stages` (names of STAGES)."""
        mode = int(bool(enable))
        if enable and stages is not None:
            mode = -sum(1 << self.STAGES.index(s) for s in stages)
        check(lib().orbx_profile_enable(self._h, mode), "orbx_profile_enable")

    def profile_read(self):
        """{stage: (total_ms, launches)} since the last read (HIP events on the launch stream)."""
        ms = np.zeros(4, np.float64)
        n = np.zeros(4, np.int32)
        check(lib().orbx_profile_read(self._h, ptr(ms), ptr(n)), "orbx_profile_read")
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.STAGES)}

    def debug_level(self, level, frame=0, stage="candidates"):
        """Per-stage diagnostics of the last extraction: (x, y, score) int arrays of the FAST
        candidates (DetectFAST order) or of the quadtree output (list order)."""
        fn = lib().orbx_debug_level_candidates if stage == "candidates" else lib().orbx_debug_level_selected
        n = C.c_int(0)
        check(fn(self._h, frame, level, None, 0, C.byref(n)), stage)
        a = np.zeros(max(n.value, 1), np.uint32)
        check(fn(self._h, frame, level, ptr(a), n.value, C.byref(n)), stage)
        a = a[:n.value]
        return np.stack([a & 0xfff, (a >> 12) & 0xfff, a >> 24], axis=1).astype(np.int32)

    # -- batched, HBM-resident mode (torch tensors on the GPU)
    def extract_batch_device(self, frames, kps_out=None, desc_out=None, counts_out=None, stream=None):
        """frames: uint8 CUDA tensor [F, H, W].  Returns (kps [F,cap,28B] as int32 view, desc [F,cap,32],
        counts [F]) — enqueued on `stream` (torch current stream by default), no host sync."""
        import torch
        assert frames.is_cuda and frames.dtype == torch.uint8 and frames.dim() == 3
        F, H, W = frames.shape
        cap = self.max_keypoints(H, W)
        dev = frames.device
        if kps_out is None:
            kps_out = torch.empty((F, cap, 7), dtype=torch.int32, device=dev)
        if desc_out is None:
            desc_out = torch.empty((F, cap, 32), dtype=torch.uint8, device=dev)
        if counts_out is None:
            counts_out = torch.empty((F,), dtype=torch.int32, device=dev)
        # caller-supplied outputs: the kernels write F x cap slots, so shapes, contiguity and device
        # are checked here (a short or strided buffer would be written out of bounds)
        for t, shape, dt in ((kps_out, (F, cap, 7), torch.int32), (desc_out, (F, cap, 32), torch.uint8)):
            if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"output slots must be contiguous {dt} {shape} on {dev}, got "
                                 f"{t.dtype} {tuple(t.shape)} on {t.device}")
        if counts_out.numel() < F or counts_out.dtype != torch.int32 or not counts_out.is_contiguous() or \
                counts_out.device != dev:
            raise ValueError("counts_out must be a contiguous int32 tensor of >= F entries on the frames' device")
        if frames.stride(2) != 1:
            raise ValueError("frames must have unit column stride (rows may be padded)")
        check(lib().orbx_extract_batch_device(self._h, tptr(frames), F, H, W, C.c_size_t(frames.stride(0)),
                                              C.c_size_t(frames.stride(1)), tptr(kps_out), tptr(desc_out),
                                              tptr(counts_out), cap, stream_ptr(stream)), "orbx_extract_batch_device")
        return kps_out, desc_out, counts_out

    def batch_status(self, stream=None) -> int:
        """Device capacity-check mask of the batches since the last call (0 = none tripped); waits
        for `stream`.  Raises OrbError when a check tripped (the batch was truncated)."""
        m = C.c_uint32(0)
        check(lib().orbx_batch_status(self._h, stream_ptr(stream), C.byref(m)), "orbx_batch_status")
        return m.value

    @staticmethod
    def kps_to_numpy(kps_i32_row):
        """Convert one frame's [cap,7] int32 keypoint tensor rows (on host) to KP_DTYPE."""
        a = np.ascontiguousarray(kps_i32_row, dtype=np.int32)
        return a.view(KP_DTYPE).reshape(-1)
