"""Convert the reference's trained Policy(W) checkpoints to small .npz fixtures.

The reference stores A2C Policy weights (examples/ball_cnn_ac3.py:109-146:
fc1 -> relu -> action_head / value_head) as torch state_dicts under
examples/stored_models/ball_state3/.  They are loaded here with
torch.load(weights_only=True) (no unpickling of code) and written as plain
float32 arrays, so tests / bench on the GPU box (which has no /root/reference)
can run the on-GPU policy rollout with the reference's own trained weights.

    python tests/golden/make_policy_fixture.py
"""
import os

import numpy as np
import torch

REF = "/root/reference/examples/stored_models/ball_state3/2layer+dropout+randpos"
SRC = {5: os.path.join(REF, "episode_1500.pth"), 10: os.path.join(REF, "window_size_10", "episode_1500.pth")}
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    for W, path in SRC.items():
        sd = torch.load(path, weights_only=True, map_location="cpu")
        arrs = {k.replace(".", "_"): v.numpy().astype(np.float32) for k, v in sd.items()}
        assert arrs["fc1_weight"].shape[1] == 4 + W * W
        out = os.path.join(HERE, f"policy_w{W}.npz")
        np.savez_compressed(out, source=os.path.relpath(path, "/root/reference"), **arrs)
        print(out, {k: v.shape for k, v in arrs.items()})


if __name__ == "__main__":
    main()
