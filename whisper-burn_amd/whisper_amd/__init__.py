"""whisper_amd -- Python binding of the Whisper model runtime (include/whisper_amd.h).

Mirrors WhisperModel::{new, encode, transcribe} (zerr0o/whisper-burn
src/model/whisper.rs) over lib/libwhisper_amd.so; every Q4 projection runs in
lib/libwq4.so.  Loud failure if the native libraries are missing.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

import wq4

LIB_PATH = os.path.join(os.path.dirname(wq4.LIB_PATH), "libwhisper_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(wq4.HEADER_PATH), "whisper_amd.h")
VARIANTS = {"large_v3": 0, "medium": 1, "tiny_test": 2}
CFG_KEYS = ["n_mels", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer", "n_text_ctx",
            "n_text_state", "n_text_head", "n_text_layer", "n_vocab", "n_lang"]
_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        wq4.lib()  # libwq4.so first (RTLD_GLOBAL)
        if not os.path.exists(LIB_PATH):
            raise wq4.WQ4Error(6, f"{LIB_PATH} not built")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        vp, c_int, c_i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        i32p = ctypes.POINTER(ctypes.c_int32)
        f32p = ctypes.POINTER(ctypes.c_float)
        L.wa_last_error.restype = ctypes.c_char_p
        L.wa_model_create_synthetic.argtypes = [c_int, c_int, ctypes.c_uint64, c_int, c_int, ctypes.POINTER(vp)]
        L.wa_model_destroy.argtypes = [vp]
        L.wa_model_destroy.restype = None
        L.wa_model_config.argtypes = [vp, i32p]
        L.wa_model_device_bytes.argtypes = [vp]
        L.wa_model_device_bytes.restype = ctypes.c_size_t
        L.wa_transcribe.argtypes = [vp, vp, c_int, c_int, c_int, c_int, i32p, i32p, vp]
        L.wa_last_timings.argtypes = [vp, f32p]
        L.wa_transcribe_batches.argtypes = [vp, vp, c_int, c_int, c_int, c_int, c_int, i32p, i32p, vp]
        L.wa_last_pipeline_stats.argtypes = [vp, f32p]
        L.wa_encode.argtypes = [vp, vp, c_int, vp, vp]
        L.wa_prompt_logits.argtypes = [vp, vp, c_int, c_int, vp, vp]
        L.wa_synth_uniform.argtypes = [ctypes.c_uint64, ctypes.c_char_p, c_i64, ctypes.c_float, ctypes.c_float, f32p]
        L.wa_profile_enable.argtypes = [vp, c_int]
        L.wa_profile_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double), c_int]
        L.wa_probe_kernels.argtypes = [vp, c_int, c_int, ctypes.POINTER(ctypes.c_double), c_int]
        L.wa_decode_group_rows.argtypes = [c_int]
        L.wa_decode_group_rows.restype = c_int
        L.wa_model_create_synthetic_ex.argtypes = [c_int, c_int, ctypes.c_uint64, c_int, c_int, c_int,
                                                   ctypes.POINTER(vp)]
        L.wa_model_weight_type.argtypes = [vp]
        L.wa_model_weight_type.restype = c_int
        L.wa_model_wide_range.argtypes = [vp]
        L.wa_model_wide_range.restype = c_int
        L.wa_model_create_from_gguf.argtypes = [c_int, ctypes.c_char_p, c_int, c_int, c_int, ctypes.POINTER(vp)]
        L.wa_gguf_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
        L.wa_gguf_close.argtypes = [vp]
        L.wa_gguf_close.restype = None
        L.wa_gguf_version.argtypes = [vp]
        L.wa_gguf_version.restype = c_int
        L.wa_gguf_tensor_count.argtypes = [vp]
        L.wa_gguf_tensor_count.restype = c_i64
        L.wa_gguf_tensor_info.argtypes = [vp, c_i64, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(c_int),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(c_int),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.wa_gguf_tensor_data.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t]
        L.wa_log_mel.argtypes = [c_int, vp, c_int, c_i64, c_i64, c_int, vp, vp]
        L.wa_mel_filterbank.argtypes = [c_int, f32p, f32p]
        L.wa_xattn_check.argtypes = [c_int, vp, vp, vp, vp, c_int, vp, c_int, c_int, c_int, c_int, c_int, vp]
        L.wa_xattn_kv_check.argtypes = [c_int, vp, vp, vp, c_int, c_int, c_int, c_int, c_int, vp]
        L.wa_transcribe_trace.argtypes = [vp, vp, c_int, c_int, c_int, c_int, i32p, i32p, vp, c_int, vp, vp]
        L.wa_encoder_attention_check.argtypes = [c_int, vp, c_int, c_int, c_int, c_int, vp]
        L.wa_self_attention_check.argtypes = [c_int, vp, vp, vp, c_int, c_int, c_int, c_int, c_int, c_int, vp]
        L.wa_logits_argmax_check.argtypes = [c_int, vp, vp, c_int, c_int, c_int, c_int, c_int, vp, vp]
        for n in ("wa_xattn_check", "wa_xattn_kv_check", "wa_transcribe_trace", "wa_encoder_attention_check", "wa_self_attention_check",
                  "wa_logits_argmax_check", "wa_log_mel", "wa_mel_filterbank", "wa_model_create_synthetic", "wa_model_config", "wa_transcribe", "wa_transcribe_batches",
                  "wa_last_pipeline_stats", "wa_last_timings", "wa_encode",
                  "wa_prompt_logits", "wa_synth_uniform", "wa_profile_enable", "wa_profile_read", "wa_probe_kernels",
                  "wa_decode_group_rows",
                  "wa_model_create_from_gguf", "wa_model_create_synthetic_ex", "wa_gguf_open", "wa_gguf_tensor_info", "wa_gguf_tensor_data"):
            getattr(L, n).restype = c_int
        _lib = L
    return _lib


def check(st: int) -> None:
    if st != 0:
        raise wq4.WQ4Error(st, lib().wa_last_error().decode(errors="replace"))


def decode_group_rows(n_clips: int) -> int:
    """Clips in the largest decode group of a transcribe batch of n_clips:
    the row count of every captured decode-step launch (wa_decode_group_rows)."""
    return int(lib().wa_decode_group_rows(n_clips))


def synth_uniform(seed: int, name: str, n: int, lo: float, hi: float) -> np.ndarray:
    out = np.empty(n, np.float32)
    check(lib().wa_synth_uniform(seed, name.encode(), n, lo, hi, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return out


def _torch():
    import torch

    return torch


MEL_FRAMES = 3000
MEL_CHUNK = 480000


def mel_filterbank(n_mels: int = 128) -> tuple[np.ndarray, np.ndarray]:
    """(filters [n_mels, 201], periodic Hann window [400]) as the product builds
    them (src/audio/mel.rs:272-320); host-only."""
    fb = np.empty((n_mels, 201), np.float32)
    win = np.empty(400, np.float32)
    f32p = ctypes.POINTER(ctypes.c_float)
    check(lib().wa_mel_filterbank(n_mels, fb.ctypes.data_as(f32p), win.ctypes.data_as(f32p)))
    return fb, win


def log_mel(audio, n_mels: int = 128, n_samples: Optional[int] = None, out=None):
    """MelSpectrogram::compute_log (src/audio/mel.rs:126-157) with the pad /
    truncate / transpose of transcribe.rs:44-76, for a batch of clips on the
    GPU.  audio: cuda f32 [B, L] (16 kHz mono; the first n_samples of each row
    are used, default L) -> cuda f32 [B, n_mels, 3000], the transcribe input."""
    torch = _torch()
    assert audio.dtype == torch.float32 and audio.is_cuda and audio.dim() == 2
    if audio.stride(1) != 1:
        audio = audio.contiguous()
    B, L = audio.shape
    n = L if n_samples is None else int(n_samples)
    if out is None:
        out = torch.empty((B, n_mels, MEL_FRAMES), device=audio.device, dtype=torch.float32)
    dev = audio.device.index if audio.device.index is not None else torch.cuda.current_device()
    check(lib().wa_log_mel(dev, ctypes.c_void_p(audio.data_ptr()), B, n, audio.stride(0), n_mels,
                           ctypes.c_void_p(out.data_ptr()),
                           ctypes.c_void_p(torch.cuda.current_stream(audio.device).cuda_stream)))
    return out


def xattn_check(q, wk_raw, wv_raw, bv, enc, Tq: int, H: int, weight_type: int = 0,
                precision: int = wq4.PREC_F16X2):
    """One decoder layer's cross-attention through the product kernels
    (wa_xattn_check): q cuda f32 [B*Tq, 64H], wk_raw / wv_raw cuda uint8 raw
    weights, bv cuda f32 [64H], enc cuda f32 [B, T, 64H] -> [B*Tq, 64H]."""
    torch = _torch()
    B, T, D = enc.shape
    out = torch.empty((B * Tq, D), device=enc.device, dtype=torch.float32)
    dev = enc.device.index if enc.device.index is not None else 0
    ptr = lambda t: ctypes.c_void_p(t.contiguous().data_ptr())
    check(lib().wa_xattn_check(dev, ptr(q), ptr(wk_raw), ptr(wv_raw), ptr(bv), weight_type, ptr(enc), B, Tq, T, H,
                               precision, ptr(out)))
    return out


def xattn_kv_check(q, k, v, Tq: int, precision: int = wq4.PREC_F16X2):
    """The few-clip cross-attention over cached K / V (wa_xattn_kv_check):
    q cuda f32 [B*Tq, 64H], k / v cuda f32 head-major [B, H, T, 64] ->
    [B*Tq, 64H] (softmax(q K^T / 8) V per head)."""
    torch = _torch()
    B, H, T, _ = k.shape
    out = torch.empty((B * Tq, 64 * H), device=k.device, dtype=torch.float32)
    dev = k.device.index if k.device.index is not None else 0
    ptr = lambda t: ctypes.c_void_p(t.contiguous().data_ptr())
    check(lib().wa_xattn_kv_check(dev, ptr(q), ptr(k), ptr(v), B, Tq, T, H, precision, ptr(out)))
    return out


def _dev(t) -> int:
    return t.device.index if t.device.index is not None else 0


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def encoder_attention_check(qkv, T: int, H: int, precision: int = wq4.PREC_F16X2):
    """Encoder self-attention through the product kernel (wa_encoder_attention_check):
    qkv cuda f32 [B*T, 3*64H] -> [B*T, 64H]."""
    torch = _torch()
    qkv = qkv.contiguous()
    B = qkv.shape[0] // T
    out = torch.empty((B * T, 64 * H), device=qkv.device, dtype=torch.float32)
    check(lib().wa_encoder_attention_check(_dev(qkv), _ptr(qkv), B, T, H, precision, _ptr(out)))
    return out


def self_attention_check(qkv, cache_k, cache_v, Tq: int, H: int, kv_len: int, precision: int = wq4.PREC_F16X2):
    """Decoder self-attention through the product kernel (wa_self_attention_check):
    qkv cuda f32 [B*Tq, 3*64H]; caches [B, H, ctx, 64] (updated in place:
    the new keys / values appended at kv_len) -> [B*Tq, 64H]."""
    torch = _torch()
    B, _, ctx, _ = cache_k.shape
    out = torch.empty((B * Tq, 64 * H), device=qkv.device, dtype=torch.float32)
    check(lib().wa_self_attention_check(_dev(qkv), _ptr(qkv.contiguous()), _ptr(cache_k), _ptr(cache_v), B, Tq, H,
                                        ctx, kv_len, precision, _ptr(out)))
    return out


def logits_argmax_check(hid, emb, step: int, precision: int = wq4.PREC_F16X2, want_logits: bool = True):
    """The decode step's fused logits + greedy pick (wa_logits_argmax_check):
    hid cuda f32 [B, D], emb cuda f32 [V, D] -> (tokens int32 [B], logits
    [B, V] as the pick saw them, or None)."""
    torch = _torch()
    B, D = hid.shape
    V = emb.shape[0]
    tok = torch.empty(B, device=hid.device, dtype=torch.int32)
    lg = torch.empty((B, V), device=hid.device, dtype=torch.float32) if want_logits else None
    check(lib().wa_logits_argmax_check(_dev(hid), _ptr(hid.contiguous()), _ptr(emb.contiguous()), B, D, V, step,
                                       precision, _ptr(tok), _ptr(lg) if lg is not None else None))
    return tok, lg


class GgufReader:
    """GgufReader (src/gguf/reader.rs): header, tensor index, tensor bytes."""

    def __init__(self, path: str):
        h = ctypes.c_void_p(None)
        check(lib().wa_gguf_open(path.encode(), ctypes.byref(h)))
        self._h = h

    @property
    def version(self) -> int:
        return lib().wa_gguf_version(self._h)

    def tensors(self) -> list[dict]:
        """File-order tensor index: name, dims (GGUF order), type, offset, nbytes."""
        out = []
        for i in range(lib().wa_gguf_tensor_count(self._h)):
            name = ctypes.create_string_buffer(512)
            nd, ty = ctypes.c_int(), ctypes.c_int()
            dims = (ctypes.c_uint64 * 8)()
            off, nb = ctypes.c_uint64(), ctypes.c_uint64()
            check(lib().wa_gguf_tensor_info(self._h, i, name, 512, ctypes.byref(nd), dims, ctypes.byref(ty),
                                            ctypes.byref(off), ctypes.byref(nb)))
            out.append({"name": name.value.decode(), "dims": list(dims[: nd.value]), "type": ty.value,
                        "offset": off.value, "nbytes": nb.value})
        return out

    def tensor_data(self, name: str) -> np.ndarray:
        info = next(t for t in self.tensors() if t["name"] == name)
        buf = np.empty(info["nbytes"], np.uint8)
        check(lib().wa_gguf_tensor_data(self._h, name.encode(), buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                         buf.size))
        return buf

    def close(self):
        if self._h and self._h.value:
            lib().wa_gguf_close(self._h)
            self._h = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WhisperModel:
    """A Whisper model resident on one MI355X: synthetic weights (default) or
    a GGUF checkpoint (WhisperModel.from_gguf, src/gguf/loader.rs)."""

    WEIGHTS = {"q4_0": 0, "f16": 1}

    def __init__(self, variant: str = "large_v3", seed: int = 1234, max_batch: int = 1, device: int = 0,
                 precision: int = wq4.PREC_F16X2, gguf_path: Optional[str] = None, weights: str = "q4_0"):
        h = ctypes.c_void_p(None)
        if gguf_path is None:
            check(lib().wa_model_create_synthetic_ex(device, VARIANTS[variant], seed, max_batch, precision,
                                                     self.WEIGHTS[weights], ctypes.byref(h)))
        else:
            check(lib().wa_model_create_from_gguf(device, gguf_path.encode(), VARIANTS[variant], max_batch,
                                                  precision, ctypes.byref(h)))
        self._h = h
        self.device = device
        self.variant = variant
        self.max_batch = max_batch
        cfg = (ctypes.c_int32 * len(CFG_KEYS))()
        check(lib().wa_model_config(h, cfg))
        self.config = dict(zip(CFG_KEYS, list(cfg)))
        self.weights = {0: "q4_0", 1: "f16"}[lib().wa_model_weight_type(h)]

    @classmethod
    def from_gguf(cls, path: str, variant: str = "large_v3", max_batch: int = 1, device: int = 0,
                  precision: int = wq4.PREC_F16X2) -> "WhisperModel":
        """load_whisper_from_gguf (src/gguf/loader.rs:26-45)."""
        return cls(variant, 0, max_batch, device, precision, gguf_path=path)

    @property
    def wide_range(self) -> bool:
        """True once a transcribe overflowed the LayerNorm fold's operand range
        and the model switched to the LayerNorm path (wa_model_wide_range >= 1)."""
        return lib().wa_model_wide_range(self._h) >= 1

    @property
    def range_tier(self) -> int:
        """0 the product path, 1 the LayerNorm path, 2 the LayerNorm path with
        every FFN on per-call operand scales, 3 also every attention output in
        f32 with its output projection on per-call operand scales
        (wa_model_wide_range)."""
        return lib().wa_model_wide_range(self._h)

    def device_bytes(self) -> int:
        return int(lib().wa_model_device_bytes(self._h))

    def _stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def transcribe(self, mel, lang_token: Optional[int] = 50259, max_tokens: int = 224, eot_stop: bool = True):
        """whisper.rs:51-128 for a batch of clips; mel: cuda f32 [B, n_mels, 3000].
        Returns a list of token-id lists (special tokens excluded)."""
        torch = _torch()
        mel = mel.contiguous()
        assert mel.dtype == torch.float32 and mel.is_cuda
        B = mel.shape[0]
        toks = np.zeros((B, max_tokens), np.int32)
        nt = np.zeros(B, np.int32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        check(lib().wa_transcribe(self._h, ctypes.c_void_p(mel.data_ptr()), B,
                                  -1 if lang_token is None else int(lang_token), max_tokens, 1 if eot_stop else 0,
                                  toks.ctypes.data_as(i32p), nt.ctypes.data_as(i32p), self._stream()))
        return [toks[b, : nt[b]].tolist() for b in range(B)]

    def transcribe_batches(self, mels, lang_token: Optional[int] = 50259, max_tokens: int = 224,
                           eot_stop: bool = True):
        """transcribe over mels cuda f32 [NB, B, n_mels, 3000], the next batch's
        encoder pipelined beside each decode (wa_transcribe_batches).  Returns
        NB lists of B token-id lists."""
        torch = _torch()
        mels = mels.contiguous()
        assert mels.dtype == torch.float32 and mels.is_cuda and mels.dim() == 4
        NB, B = mels.shape[0], mels.shape[1]
        toks = np.zeros((NB, B, max_tokens), np.int32)
        nt = np.zeros((NB, B), np.int32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        check(lib().wa_transcribe_batches(self._h, ctypes.c_void_p(mels.data_ptr()), NB, B,
                                          -1 if lang_token is None else int(lang_token), max_tokens,
                                          1 if eot_stop else 0, toks.ctypes.data_as(i32p), nt.ctypes.data_as(i32p),
                                          self._stream()))
        return [[toks[i, b, : nt[i, b]].tolist() for b in range(B)] for i in range(NB)]

    def pipeline_stats(self) -> dict:
        """After transcribe_batches: batches, mean encoder layers run beside a
        decode, mean ms of that CU-masked part, CUs of the masked stream."""
        t = (ctypes.c_float * 4)()
        check(lib().wa_last_pipeline_stats(self._h, t))
        return {"batches": int(t[0]), "overlap_layers": t[1], "masked_ms": t[2], "masked_cus": int(t[3])}

    def transcribe_trace(self, mel, trace_ids: np.ndarray, lang_token: Optional[int] = 50259,
                         max_tokens: int = 224, eot_stop: bool = False):
        """transcribe + the decode-step logit trace (wa_transcribe_trace):
        trace_ids int32 [B, max_tokens + 1, K] -> (tokens, logits [B,
        max_tokens + 1, K] float32; slot 0 and slots past a clip's last step
        are NaN)."""
        torch = _torch()
        mel = mel.contiguous()
        B = mel.shape[0]
        K = trace_ids.shape[-1]
        assert trace_ids.shape == (B, max_tokens + 1, K)
        ids = torch.from_numpy(np.ascontiguousarray(trace_ids, np.int32)).to(mel.device)
        out = torch.full((B, max_tokens + 1, K), float("nan"), device=mel.device, dtype=torch.float32)
        toks = np.zeros((B, max_tokens), np.int32)
        nt = np.zeros(B, np.int32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        check(lib().wa_transcribe_trace(self._h, _ptr(mel), B, -1 if lang_token is None else int(lang_token),
                                        max_tokens, 1 if eot_stop else 0, toks.ctypes.data_as(i32p),
                                        nt.ctypes.data_as(i32p), _ptr(ids), K, _ptr(out), self._stream()))
        return [toks[b, : nt[b]].tolist() for b in range(B)], out.cpu().numpy()

    def transcribe_audio(self, audio, lang_token: Optional[int] = 50259, max_tokens: int = 224,
                         eot_stop: bool = True, n_samples: Optional[int] = None):
        """src/transcribe.rs:34-107 from 16 kHz samples (cuda f32 [B, L]) to
        token ids: GPU log-mel (log_mel) then transcribe."""
        mel = log_mel(audio, self.config["n_mels"], n_samples)
        return self.transcribe(mel, lang_token, max_tokens, eot_stop)

    def last_timings(self) -> dict:
        t = (ctypes.c_float * 5)()
        check(lib().wa_last_timings(self._h, t))
        return {"encoder_ms": t[0], "cross_kv_ms": t[1], "prompt_ms": t[2], "decode_ms": t[3], "steps": int(t[4])}

    PROF_NAMES = ("q4_gemm", "encoder_attention", "conv", "layernorm")

    def profile_enable(self, on: bool = True) -> None:
        check(lib().wa_profile_enable(self._h, 1 if on else 0))

    def profile_read(self, reset: bool = True) -> dict:
        """Per category: launches, ms, algorithmic GFLOP and GB (HIP events)."""
        buf = (ctypes.c_double * 16)()
        check(lib().wa_profile_read(self._h, buf, 1 if reset else 0))
        return {n: {"launches": int(buf[4 * i]), "ms": buf[4 * i + 1], "gflop": buf[4 * i + 2], "gb": buf[4 * i + 3]}
                for i, n in enumerate(self.PROF_NAMES)}

    def probe_kernels(self, n_clips: int, iters: int = 20) -> dict:
        """HIP-event timing of single decode-step kernels (after transcribe)."""
        buf = (ctypes.c_double * 6)()
        check(lib().wa_probe_kernels(self._h, n_clips, iters, buf, len(buf)))
        return {"cross_attention": {"us": buf[0], "bytes": buf[1], "kv_cache": buf[5] != 0.0},
                "decode_fc1": {"us": buf[2], "bytes": buf[3], "flops": buf[4]}}

    def encode(self, mel):
        """encoder.rs:87-115 -> encoder_out [B, 1500, D] (also writes the f16 encoder-output planes the decoder cross-attention reads)."""
        torch = _torch()
        B = mel.shape[0]
        out = torch.empty((B, self.config["n_audio_ctx"], self.config["n_audio_state"]), device=mel.device,
                          dtype=torch.float32)
        check(lib().wa_encode(self._h, ctypes.c_void_p(mel.contiguous().data_ptr()), B,
                              ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def prompt_logits(self, prompt):
        """decoder.rs:251-296 after encode(): prompt int32 cuda [B, T<=4] -> last-position logits."""
        torch = _torch()
        B, T = prompt.shape
        out = torch.empty((B, self.config["n_vocab"]), device=prompt.device, dtype=torch.float32)
        check(lib().wa_prompt_logits(self._h, ctypes.c_void_p(prompt.contiguous().data_ptr()), B, T,
                                     ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def close(self):
        if self._h and self._h.value:
            lib().wa_model_destroy(self._h)
            self._h = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
