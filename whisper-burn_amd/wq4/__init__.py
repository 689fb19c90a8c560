"""wq4 -- Python host mirror of the reference's Q4 operator surface.

Mirrors zerr0o/whisper-burn src/gguf/{tensor,op,linear}.rs and
src/model/layers.rs (Q4FFN, gelu) over the C ABI in include/wq4.h
(libwq4.so, hand-written HIP kernels for gfx950).  PyTorch is used only as
device-memory / stream plumbing: activations are torch tensors on `cuda:N`,
their data pointers and the current HIP stream are handed to the C ABI.

There is no fallback: if lib/libwq4.so is missing or cannot be loaded every
entry point raises ``WQ4Error`` -- the product never computes on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Optional, Sequence

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# WQ4_LIB_DIR: load the libraries from another build directory (the timing
# diagnostics: `scripts/gpu.sh libs` / WQ4_LIB_DIR); the product build is lib/.
LIB_PATH = os.path.join(os.environ.get("WQ4_LIB_DIR") or os.path.join(_PKG_ROOT, "lib"), "libwq4.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG_ROOT), "include", "wq4.h")

WQ4_OK = 0
STATUS_NAMES = {0: "WQ4_OK", 1: "WQ4_EINVAL", 2: "WQ4_ESHAPE", 3: "WQ4_EBYTES", 4: "WQ4_EHIP", 5: "WQ4_ENOMEM",
                6: "WQ4_EUNSUPPORTED", 7: "WQ4_ERANGE"}
PREC_F16X2 = 0
PREC_F16 = 1
EPI_GELU = 1
EPI_RESIDUAL = 2


class WQ4Error(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status
        self.msg = msg


_lib: Optional[ctypes.CDLL] = None


def _declare(L: ctypes.CDLL) -> None:
    c_int, c_i64, c_sz, vp = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p
    u8p = ctypes.POINTER(ctypes.c_uint8)
    f32p = ctypes.POINTER(ctypes.c_float)
    L.wq4_last_error.restype = ctypes.c_char_p
    L.wq4_abi_version.restype = c_int
    L.wq4_device_count.argtypes = [ctypes.POINTER(c_int)]
    L.wq4_set_precision.argtypes = [c_int]
    L.wq4_get_precision.restype = c_int
    L.wq4_set_kernel_policy.argtypes = [c_int]
    L.wq4_gemm_kernel_name.argtypes = [c_i64, c_i64, c_i64]
    L.wq4_gemm_kernel_name.restype = ctypes.c_char_p
    L.wq4_tensor_create.argtypes = [c_int, u8p, c_sz, c_i64, c_i64, ctypes.POINTER(vp)]
    L.wq4_tensor_destroy.argtypes = [vp]
    L.wq4_tensor_destroy.restype = None
    L.wq4_tensor_shape.argtypes = [vp, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]
    L.wq4_tensor_num_blocks.argtypes = [vp]
    L.wq4_tensor_num_blocks.restype = c_i64
    L.wq4_tensor_device.argtypes = [vp]
    L.wq4_tensor_device.restype = c_int
    L.wq4_tensor_device_bytes.argtypes = [vp]
    L.wq4_tensor_device_bytes.restype = c_sz
    L.wq4_tensor_dequantize.argtypes = [vp, f32p]
    L.wq4_tensor_raw_bytes.argtypes = [vp, u8p]
    L.wq4_matmul.argtypes = [vp, vp, vp, c_i64, c_i64, c_i64, vp]
    L.wq4_linear_forward.argtypes = [vp, vp, vp, vp, c_i64, c_i64, c_i64, vp]
    L.wq4_ffn_forward.argtypes = [vp, vp, vp, vp, vp, vp, c_i64, c_i64, vp]
    L.wq4_linear_workspace_bytes.argtypes = [vp, c_i64]
    L.wq4_linear_workspace_bytes.restype = c_sz
    L.wq4_ffn_workspace_bytes.argtypes = [vp, vp, c_i64]
    L.wq4_ffn_workspace_bytes.restype = c_sz
    L.wq4_linear_forward_ws.argtypes = [vp, vp, vp, vp, vp, c_i64, c_i64, ctypes.c_uint, c_int, vp, c_sz, vp]
    L.wq4_ffn_forward_ws.argtypes = [vp, vp, vp, vp, vp, vp, vp, c_i64, ctypes.c_uint, c_int, vp, c_sz, vp]
    L.wq4_debug_repack.argtypes = [u8p, c_i64, c_i64, u8p, ctypes.POINTER(ctypes.c_uint32), f32p]
    L.wq4_quantize_q4_0.argtypes = [f32p, c_i64, u8p]
    L.wq4_tensor_create_f16.argtypes = [c_int, ctypes.POINTER(ctypes.c_uint16), c_i64, c_i64, ctypes.POINTER(vp)]
    L.wq4_tensor_create_ex.argtypes = [c_int, u8p, c_sz, c_i64, c_i64, ctypes.c_uint, ctypes.POINTER(vp)]
    L.wq4_tensor_create_f16_ex.argtypes = [c_int, ctypes.POINTER(ctypes.c_uint16), c_i64, c_i64, ctypes.c_uint,
                                           ctypes.POINTER(vp)]
    L.wq4_debug_set_enc_kernel.argtypes = [c_int]
    L.wq4_debug_set_enc_kernel.restype = c_int
    L.wq4_tensor_has_decode_step.argtypes = [vp]
    L.wq4_tensor_has_decode_step.restype = c_int
    L.wq4_tensor_weight_type.argtypes = [vp]
    L.wq4_tensor_weight_type.restype = c_int
    L.wq4_debug_unrepack.argtypes = [u8p, ctypes.POINTER(ctypes.c_uint32), f32p, c_i64, c_i64, u8p]
    L.wq4_debug_repacked_bytes.argtypes = [c_i64, c_i64, ctypes.POINTER(c_sz), ctypes.POINTER(c_sz),
                                           ctypes.POINTER(c_sz)]
    L.wq4_atiled_bytes.argtypes = [c_i64, c_i64, c_int]
    L.wq4_atiled_bytes.restype = c_sz
    L.wq4_tile_activations.argtypes = [vp, c_i64, c_i64, c_i64, c_int, vp, c_sz, vp]
    L.wq4_linear_forward_tiled.argtypes = [vp, vp, vp, vp, vp, c_i64, ctypes.c_uint, c_int, vp]
    L.wq4_linear_forward_tiled_out.argtypes = [vp, vp, vp, vp, c_sz, c_i64, ctypes.c_uint, c_int, vp]
    L.wq4_gemm_tiled.argtypes = [vp, vp, vp, vp, vp, vp, c_i64, ctypes.c_uint, c_int, c_int, vp]
    L.wq4_gemm_tiled_headmajor.argtypes = [vp, vp, vp, vp, c_i64, c_int, c_int, c_int, c_int, vp]
    L.wq4_layernorm.argtypes = [vp, vp, vp, c_i64, c_i64, c_int, vp, vp, vp]
    L.wq4_prepare_stream.argtypes = [c_int, vp]
    L.wq4_gemm_ln_tiled.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, c_i64, ctypes.c_uint, c_int, c_int, vp]
    L.wq4_gemm_tiled_lnfold.argtypes = [vp, vp, vp, vp, vp, vp, c_i64, ctypes.c_uint, c_int, ctypes.POINTER(LnFold), vp]
    L.wq4_ln_fold_vectors.argtypes = [vp, f32p, f32p, f32p, f32p, f32p]
    L.wq4_lnfold_supported.argtypes = [vp, c_i64]
    for name in ("wq4_gemm_tiled_lnfold", "wq4_ln_fold_vectors", "wq4_lnfold_supported", "wq4_gemm_ln_tiled", "wq4_tile_activations", "wq4_linear_forward_tiled", "wq4_linear_forward_tiled_out", "wq4_gemm_tiled",
                 "wq4_gemm_tiled_headmajor", "wq4_layernorm", "wq4_prepare_stream"):
        getattr(L, name).restype = c_int
    for name in ("wq4_device_count", "wq4_set_precision", "wq4_set_kernel_policy", "wq4_tensor_create",
                 "wq4_tensor_shape", "wq4_tensor_dequantize", "wq4_tensor_raw_bytes", "wq4_matmul",
                 "wq4_linear_forward", "wq4_ffn_forward", "wq4_linear_forward_ws", "wq4_ffn_forward_ws",
                 "wq4_debug_repack", "wq4_debug_unrepack", "wq4_debug_repacked_bytes", "wq4_quantize_q4_0", "wq4_tensor_create_f16",
                 "wq4_tensor_create_ex", "wq4_tensor_create_f16_ex"):
        getattr(L, name).restype = c_int


class LnFold(ctypes.Structure):
    """wq4_ln_fold (include/wq4.h): LayerNorm folded into the GEMMs around it."""
    _fields_ = [("gamma_dev", ctypes.c_void_p), ("at_out_dev", ctypes.c_void_p), ("stats_out_dev", ctypes.c_void_p),
                ("stats_in_dev", ctypes.c_void_p), ("wg_dev", ctypes.c_void_p)]


def lib() -> ctypes.CDLL:
    """Load lib/libwq4.so (RTLD_GLOBAL so the model library can link to it)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise WQ4Error(6, f"{LIB_PATH} not built (run __graft_entry__.build() or make -C whisper-burn_amd)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _declare(L)
        _lib = L
    return _lib


def check(status: int) -> None:
    if status != WQ4_OK:
        raise WQ4Error(status, lib().wq4_last_error().decode(errors="replace"))


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Every function declared in include/wq4.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wq4_[a-z0-9_]+)\s*\(", text)))


def device_count() -> int:
    n = ctypes.c_int(0)
    st = lib().wq4_device_count(ctypes.byref(n))
    return n.value if st == WQ4_OK else 0


def set_precision(prec: int) -> None:
    check(lib().wq4_set_precision(prec))


def get_precision() -> int:
    return lib().wq4_get_precision()


def set_kernel_policy(policy: int) -> None:
    """0 = automatic, 1 = MFMA tile ("prefill") kernel, 2 = K-split ("decode")
    kernel, 3 = decode-step kernel (include/wq4.h)."""
    check(lib().wq4_set_kernel_policy(policy))


def gemm_kernel_name(n: int, k: int, rows: int) -> str:
    """The kernel a Q4_0 GEMM of `rows` rows over [n, k] weights runs under the
    current policy (host only; include/wq4.h wq4_gemm_kernel_name)."""
    return lib().wq4_gemm_kernel_name(n, k, rows).decode()


def _u8p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _f32p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def quantize_q4_0(x: np.ndarray) -> np.ndarray:
    """Q4_0 bytes of f32 values (scripts/convert_whisper.py:33-74 semantics)."""
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    out = np.empty(x.size // 32 * 18, np.uint8)
    check(lib().wq4_quantize_q4_0(_f32p(x), x.size, _u8p(out)))
    return out


def debug_repack(raw: np.ndarray, n: int, k: int) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Host-only: the upload repack (wq4_layout.cpp) without touching a GPU.
    Returns (nibbles u8, scales u32 = 2 x f16 d', column scales f32)."""
    nb, sb, cb = ctypes.c_size_t(0), ctypes.c_size_t(0), ctypes.c_size_t(0)
    check(lib().wq4_debug_repacked_bytes(n, k, ctypes.byref(nb), ctypes.byref(sb), ctypes.byref(cb)))
    raw = np.ascontiguousarray(raw, np.uint8)
    nib = np.zeros(nb.value, np.uint8)
    sc = np.zeros(sb.value // 4, np.uint32)
    cs = np.zeros(cb.value // 4, np.float32)
    check(lib().wq4_debug_repack(_u8p(raw), n, k, _u8p(nib), sc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                 _f32p(cs)))
    return nib, sc, cs


def debug_unrepack(nib: np.ndarray, sc: np.ndarray, cs: np.ndarray, n: int, k: int) -> np.ndarray:
    out = np.zeros(n * k // 32 * 18, np.uint8)
    check(lib().wq4_debug_unrepack(_u8p(np.ascontiguousarray(nib, np.uint8)),
                                   np.ascontiguousarray(sc, np.uint32).ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                   _f32p(np.ascontiguousarray(cs, np.float32)), n, k, _u8p(out)))
    return out


# ----------------------------------------------------------------------------
# Reference-shaped API (src/gguf/tensor.rs, op.rs, linear.rs; layers.rs)
# ----------------------------------------------------------------------------
def _torch():
    import torch  # plumbing only: device memory + streams

    return torch


def _stream_ptr(device_index: int):
    torch = _torch()
    return ctypes.c_void_p(torch.cuda.current_stream(device_index).cuda_stream)


def _dev_ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)


class Q4Tensor:
    """A Q4_0 weight tensor resident on an MI355X (src/gguf/tensor.rs:21-113)."""

    def __init__(self, handle: ctypes.c_void_p, shape: tuple[int, int], device: int):
        self._h = handle
        self._shape = shape
        self._device = device

    @classmethod
    def from_q4_bytes(cls, raw_bytes, shape: Sequence[int], device: int = 0,
                      decode_step: bool = True) -> "Q4Tensor":
        """tensor.rs:35-71.  Raises WQ4Error(WQ4_ESHAPE / WQ4_EBYTES) with the
        reference's messages on bad input.  decode_step=False skips the
        <= 32-row kernel's second weight copy (WQ4_TENSOR_NO_DECODE_STEP)."""
        n, k = int(shape[0]), int(shape[1])
        raw = np.ascontiguousarray(np.frombuffer(bytes(raw_bytes), np.uint8) if isinstance(raw_bytes, (bytes, bytearray))
                                   else np.asarray(raw_bytes, np.uint8)).ravel()
        h = ctypes.c_void_p(None)
        check(lib().wq4_tensor_create_ex(device, _u8p(raw), raw.size, n, k, 0 if decode_step else 1, ctypes.byref(h)))
        return cls(h, (n, k), device)

    @classmethod
    def from_f16(cls, weights, device: int = 0, decode_step: bool = True) -> "Q4Tensor":
        """Unquantized f16 weights [N, K] (BASELINE config 5): the same GEMM
        entry points run on them (wq4_tensor_create_f16)."""
        w = np.ascontiguousarray(np.asarray(weights), dtype=np.float16)
        n, k = w.shape
        h = ctypes.c_void_p(None)
        check(lib().wq4_tensor_create_f16_ex(device, w.view(np.uint16).ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
                                             n, k, 0 if decode_step else 1, ctypes.byref(h)))
        return cls(h, (n, k), device)

    @property
    def has_decode_step(self) -> bool:
        """True if the <= 32-row (decode-step) kernel's weight layout exists."""
        return bool(lib().wq4_tensor_has_decode_step(self._h))

    @property
    def weight_type(self) -> str:
        return {0: "q4_0", 1: "f16"}[lib().wq4_tensor_weight_type(self._h)]

    def shape(self) -> list[int]:
        """tensor.rs:74-76 -> [N, K]."""
        return [self._shape[0], self._shape[1]]

    def num_blocks(self) -> int:
        """tensor.rs:79-81."""
        return int(lib().wq4_tensor_num_blocks(self._h))

    @property
    def device(self) -> int:
        return self._device

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def device_bytes(self) -> int:
        return int(lib().wq4_tensor_device_bytes(self._h))

    def dequantize_host(self) -> np.ndarray:
        n, k = self._shape
        out = np.empty(n * k, np.float32)
        check(lib().wq4_tensor_dequantize(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        return out.reshape(n, k)

    def dequantize(self):
        """tensor.rs:88-113: D2H read, host dequant, returned as a device tensor."""
        torch = _torch()
        return torch.from_numpy(self.dequantize_host()).to(f"cuda:{self._device}")

    def raw_bytes(self) -> np.ndarray:
        n, k = self._shape
        out = np.empty(n * k * 2 if self.weight_type == "f16" else n * k // 32 * 18, np.uint8)
        check(lib().wq4_tensor_raw_bytes(self._h, _u8p(out)))
        return out

    def close(self) -> None:
        if self._h and self._h.value:
            lib().wq4_tensor_destroy(self._h)
            self._h = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _check_input(x, w: Q4Tensor):
    torch = _torch()
    if x.dim() != 3:  # op.rs:53
        raise WQ4Error(2, "Input must be 3D [B, M, K]")
    if x.dtype != torch.float32 or not x.is_cuda:
        raise WQ4Error(1, "input must be a float32 cuda tensor")
    if x.device.index != w.device:
        raise WQ4Error(1, f"input on cuda:{x.device.index}, weights on cuda:{w.device}")
    return x.contiguous()  # op.rs:50 (into_contiguous)


def q4_matmul(x, weights: Q4Tensor):
    """op.rs:47-117: out[B,M,N] = x[B,M,K] . W[N,K]^T (fresh f32 output)."""
    torch = _torch()
    x = _check_input(x, weights)
    b, m, k = x.shape
    n = weights.shape()[0]
    out = torch.empty((b, m, n), dtype=torch.float32, device=x.device)
    check(lib().wq4_matmul(weights.handle, _dev_ptr(x), _dev_ptr(out), b, m, k, _stream_ptr(weights.device)))
    return out


class Q4Linear:
    """src/gguf/linear.rs:17-40 -- x @ W^T + bias (bias fused in the epilogue)."""

    def __init__(self, weights: Q4Tensor, bias=None):
        self.weights = weights
        self.bias = None if bias is None else bias.contiguous().float()

    def forward(self, x):
        torch = _torch()
        x = _check_input(x, self.weights)
        b, m, k = x.shape
        n = self.weights.shape()[0]
        out = torch.empty((b, m, n), dtype=torch.float32, device=x.device)
        check(lib().wq4_linear_forward(self.weights.handle, _dev_ptr(self.bias), _dev_ptr(x), _dev_ptr(out), b, m, k,
                                       _stream_ptr(self.weights.device)))
        return out

    __call__ = forward


class Q4FFN:
    """src/model/layers.rs:44-58 -- fc2(gelu(fc1(x))) in two fused launches."""

    def __init__(self, fc1: Q4Linear, fc2: Q4Linear):
        self.fc1 = fc1
        self.fc2 = fc2

    def forward(self, x):
        torch = _torch()
        x = _check_input(x, self.fc1.weights)
        b, m, d = x.shape
        if self.fc1.weights.shape()[1] != d:
            raise WQ4Error(2, f"K dimension mismatch: input has {d}, weights have {self.fc1.weights.shape()[1]}")
        out = torch.empty((b, m, self.fc2.weights.shape()[0]), dtype=torch.float32, device=x.device)
        check(lib().wq4_ffn_forward(self.fc1.weights.handle, _dev_ptr(self.fc1.bias), self.fc2.weights.handle,
                                    _dev_ptr(self.fc2.bias), _dev_ptr(x), _dev_ptr(out), b, m,
                                    _stream_ptr(self.fc1.weights.device)))
        return out

    __call__ = forward
