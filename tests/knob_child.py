"""Child process of test_tuning_knobs_gpu.py: the environment knobs are read
once per process (static initialisers), so every setting runs in its own
interpreter.  Prints the greedy tokens of 16 synthetic tiny_test clips as
one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(REPO, "oracle"), os.path.join(REPO, "whisper-burn_amd"),
                os.path.join(REPO, "whisper-burn_amd", "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import whisper_amd  # noqa: E402
import whisper_oracle as wo  # noqa: E402

mel = np.stack([wo.synthetic_mel(20 + c, 80) for c in range(16)]).astype(np.float32)
m = whisper_amd.WhisperModel("tiny_test", 1234, max_batch=16)
tok = m.transcribe(torch.from_numpy(mel).cuda(), 50259, max_tokens=24)
m.close()
print(json.dumps(tok))
