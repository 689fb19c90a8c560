"""Standalone decode-step logits + pick (wa_logits_argmax_check) at the
large-v3 shape, REPS calls, for rocprofv3 --kernel-trace: the kernel's
duration alone (in the model it shares the chip with the other decode
group).  B (clips) from the env, default 16 = one of two decode groups."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "whisper-burn_amd"))
import whisper_amd  # noqa: E402

B = int(os.environ.get("B", "16"))
REPS = int(os.environ.get("REPS", "20"))
D, V = 1280, 51866
g = torch.Generator().manual_seed(0)
hid = torch.randn(B, D, generator=g).cuda()
emb = (torch.randn(V, D, generator=g) * 0.02).cuda()
for _ in range(REPS):
    tok, _ = whisper_amd.logits_argmax_check(hid, emb, 5, want_logits=False)
torch.cuda.synchronize()
print("tokens", tok[:4].tolist())
