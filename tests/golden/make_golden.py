"""Generate tests/golden/q4_golden.npz from the REFERENCE's own quantizer.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):

    python tests/golden/make_golden.py

It imports /root/reference/scripts/convert_whisper.py by path (its top-level
imports are argparse/struct/numpy/pathlib only; convert_model(), which would
download a model by name, is never called) and records, for each input array,
the exact bytes that `quantize_q4_0` (convert_whisper.py:33-74) produces under
this container's numpy (2.2.6).  The fixture holds data only: inputs and
expected outputs.  No reference source is copied into the repository.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SCRIPT = "/root/reference/scripts/convert_whisper.py"

sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402  (closed-form inputs from the C restatement)


def load_reference_quantizer():
    spec = importlib.util.spec_from_file_location("ref_convert_whisper", REF_SCRIPT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def cases() -> dict[str, np.ndarray]:
    rng = np.random.default_rng(20260227)
    c: dict[str, np.ndarray] = {}
    # known-answer inputs of src/gguf/tests.rs
    c["ramp_pm1"] = ((np.arange(32, dtype=np.float32) - np.float32(15.5)) / np.float32(15.5)).astype(np.float32)  # :193
    c["zeros"] = np.zeros(32, np.float32)  # :231
    c["uniform_half"] = np.full(32, 0.5, np.float32)  # :239
    c["large"] = ((np.arange(32, dtype=np.float32) - np.float32(15.5)) * np.float32(100.0)).astype(np.float32)  # :253
    c["gguf_sin_32x64"] = oracle.closed_form(6, 32 * 64)  # :283
    c["const_0p1_1024"] = np.full(1024, 0.1, np.float32)  # :306
    c["const_0p2_2048"] = np.full(2048, 0.2, np.float32)  # :307
    c["const_m0p1_2048"] = np.full(2048, -0.1, np.float32)  # :308
    c["dq_16x16"] = oracle.closed_form(4, 256)  # :337
    c["small_w_32x32"] = oracle.closed_form(2, 32 * 32)  # :377
    c["shape_w_64x128"] = oracle.closed_form(1, 64 * 128)  # :436 (first shape)
    c["shape_w_1280x1280_rows0_63"] = oracle.closed_form(1, 64 * 1280)  # :436 (first 64 rows)
    c["linear_w_64x128"] = oracle.closed_form(0, 64 * 128)  # :493
    c["bias_w_32x64"] = oracle.closed_form(0, 32 * 64)  # :515
    c["ffn_w_256x64"] = oracle.closed_form(7, 256 * 64)  # :580
    c["roundtrip_32x64"] = oracle.closed_form(5, 32 * 64)  # :669
    # rounding ties: amax = 7 -> d = 1 exactly, values at k + 0.5 (half-to-even)
    ties = np.array([7.0, -7.0] + [k + 0.5 for k in range(-7, 7)] * 2 + [0.5, -0.5], np.float32)
    c["ties_d1"] = ties
    # f16 scale edge cases: subnormal scale, scale rounding to zero, huge scale
    c["tiny_subnormal_scale"] = (rng.standard_normal(32 * 16) * 1e-6).astype(np.float32)
    c["tiny_zero_scale"] = (rng.standard_normal(32 * 4) * 1e-9).astype(np.float32)
    c["huge"] = (rng.standard_normal(32 * 8) * 2.0e4).astype(np.float32)
    c["sparse_one_hot"] = np.zeros(32 * 8, np.float32)
    c["sparse_one_hot"][::37] = 1.0
    # random weights at Whisper-like scales
    for s in (0.02, 0.05, 1.0):
        c[f"normal_{s}"] = (rng.standard_normal(32 * 4096) * s).astype(np.float32)
    c["uniform_pm1"] = rng.uniform(-1, 1, 32 * 4096).astype(np.float32)
    return c


def main() -> None:
    ref = load_reference_quantizer()
    out: dict[str, np.ndarray] = {}
    for name, x in cases().items():
        q = np.frombuffer(ref.quantize_q4_0(x), np.uint8).copy()
        out[f"in/{name}"] = x
        out[f"q4/{name}"] = q
    # the reference's tensor-selection rule, as data (convert_whisper.py:77-96)
    names = ["encoder.blocks.0.attn.query.weight", "encoder.blocks.0.attn.query.bias",
             "encoder.blocks.0.mlp.0.weight", "decoder.token_embedding.weight",
             "encoder.positional_embedding", "encoder.conv1.weight", "decoder.blocks.3.cross_attn_ln.weight",
             "decoder.blocks.3.cross_attn.key.weight", "tiny.weight"]
    shapes = [(1280, 1280), (1280,), (5120, 1280), (51866, 1280), (1500, 1280), (1280, 128, 3), (1280,),
              (1280, 1280), (128, 255)]
    sel = np.array([bool(ref.should_quantize(n, s)) for n, s in zip(names, shapes)])
    out["select/names"] = np.array(names)
    out["select/quantize"] = sel
    # the reference HF->GGUF name map (convert_whisper.py:224-275), as data
    hf = ["model.encoder.layers.3.self_attn.q_proj.weight", "model.encoder.layers.3.fc1.weight",
          "model.encoder.layer_norm.weight", "model.encoder.embed_positions.weight",
          "model.decoder.layers.0.encoder_attn.k_proj.weight", "model.decoder.layers.0.encoder_attn_layer_norm.bias",
          "model.decoder.embed_tokens.weight", "model.decoder.layers.5.fc2.bias",
          "model.encoder.conv1.weight", "model.decoder.layer_norm.bias"]
    out["names/hf"] = np.array(hf)
    out["names/gguf"] = np.array([ref.hf_name_to_gguf(h) for h in hf])
    out["meta/numpy_version"] = np.array(np.__version__)
    path = os.path.join(HERE, "q4_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
