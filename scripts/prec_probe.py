"""Full-size fixtures (tests/golden/full_*.npz) run at another model
precision: token flips against the f32 oracle (with the oracle's top-2
margin at each flip) and the worst decode-logit error as a fraction of
tests/test_full_size_gpu.py's f64-derived bound.  Evidence for the precision
choice, not a test.   python3 scripts/prec_probe.py [f16|f16x2]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper-burn_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import whisper_amd  # noqa: E402
import wq4  # noqa: E402
from test_full_size_gpu import CASES, _bound, _fixture  # noqa: E402
from whisper_oracle import synthetic_mel  # noqa: E402

prec = {"f16": wq4.PREC_F16, "f16x2": wq4.PREC_F16X2}[sys.argv[1] if len(sys.argv) > 1 else "f16"]
out = {}
for name in CASES:
    f, meta = _fixture(name)
    clips, steps, lang = meta["clips"], meta["steps"], meta["lang"]
    B = len(clips)
    m = whisper_amd.WhisperModel(meta["variant"], meta["seed"], max_batch=B, weights=meta["weights"], precision=prec)
    mel = torch.from_numpy(np.stack([synthetic_mel(c, m.config["n_mels"]) for c in clips])).cuda()
    toks, lg = m.transcribe_trace(mel, f["top_ids"], lang, steps, eot_stop=False)
    ref = f["tokens_f32"]
    flips = [(b, s, float(f["margin_f32"][b, s])) for b in range(B) for s in range(steps) if toks[b][s] != ref[b, s]]
    first = min((s for _, s, _ in flips), default=None)
    # logit error before the first flip (after it the sequences differ)
    got = lg[:, 1:, :].astype(np.float64)
    r32, r64 = f["top_f32"][:, 1:, :], f["top_f64"][:, 1:, :]
    worst = 0.0
    for b in range(B):
        for s in range(steps if first is None else first):
            k = np.isfinite(r64[b, s])
            worst = max(worst, float(np.max(np.abs(got[b, s, k] - r64[b, s, k]))) / _bound(r32[b, s, k], r64[b, s, k]))
    out[name] = {"flips": len(flips), "first_flip_step": first, "first_flip_margin": flips[0][2] if flips else None,
                 "worst_logit_err_over_bound_before_flip": round(worst, 3)}
    print(name, out[name], flush=True)
    m.close()
json.dump(out, open(os.path.join(REPO, "gpurun_out", f"prec_probe_{sys.argv[1] if len(sys.argv) > 1 else 'f16'}.json"), "w"), indent=1)
