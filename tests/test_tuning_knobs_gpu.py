"""The product's environment tuning knobs, each run end to end (GPU).

Every knob only re-plans work the default path already does -- the
LayerNorm fold off (wa_model.cpp lnfold_on: WA_LN_FOLD),
another number of decode groups (wa_model.cpp decode_groups:
WA_DECODE_GROUPS) or the cross-attention over cached K / V for more clips
(wa_model.cpp kv_config: WA_XATTN_KV_CLIPS, whose groups then also form
their qkv / query projections inside the attention launches) -- so the greedy tokens of 16 synthetic tiny_test clips
must equal the default's, and a sample must equal the oracle's
(oracle/whisper_oracle.py).  The knobs are read once per process, so each
setting runs tests/knob_child.py in a child interpreter.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

import whisper_oracle as wo

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KNOBS = [
    {},
    {"WQ4_KERNEL_POLICY": "3"},                           # every <= 32-row GEMM on the decode-step kernel
    {"WA_LN_FOLD": "0"},                                  # LayerNorm as its own pass
    {"WA_DECODE_GROUPS": "1"},
    {"WA_DECODE_GROUPS": "3"},                            # ragged groups 6/5/5
    {"WA_XATTN_KV_CLIPS": "16"},                          # cross K/V caches, two groups of 8
    {"WA_XATTN_KV_CLIPS": "16", "WA_DECODE_GROUPS": "3"},  # ... at ragged group offsets
]


def _run(env_over):
    env = dict(os.environ)
    for k in ("WQ4_KERNEL_POLICY", "WA_LN_FOLD",
              "WA_DECODE_GROUPS", "WA_XATTN_KV_CLIPS"):
        env.pop(k, None)
    env.update(env_over)
    r = subprocess.run([sys.executable, os.path.join(HERE, "knob_child.py")], env=env, capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, (env_over, r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_tokens():
    return _run({})


@pytest.fixture(scope="module")
def oracle_sample():
    mel = np.stack([wo.synthetic_mel(20 + c, 80) for c in range(16)]).astype(np.float32)
    sample = [0, 5, 10, 15]
    return sample, wo.SynthWhisper("tiny_test", 1234).transcribe(mel[sample], 50259, max_tokens=24)


@pytest.mark.parametrize("knobs", KNOBS[1:], ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_knob_tokens_equal_default_and_oracle(knobs, default_tokens, oracle_sample):
    got = _run(knobs)
    assert got == default_tokens
    sample, ref = oracle_sample
    assert [got[i] for i in sample] == ref


def test_default_matches_oracle(default_tokens, oracle_sample):
    sample, ref = oracle_sample
    assert [default_tokens[i] for i in sample] == ref
