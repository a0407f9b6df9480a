"""Export the reference's pretrained ECO BA-200 network (experiments/pretrained_agent/networks/eco/
network_best_BA_200spin.pth, MIT) as plain arrays: tests/golden/pretrained_ba200.npz, the yardstick of
tests/test_training_quality_ba200_gpu.py.  Run in the build container only (needs /root/reference):
    python tests/golden/make_pretrained.py
The state_dict is read with torch.load(..., weights_only=True); no reference code is imported or run."""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    sd = torch.load(os.path.join(REF, "experiments/pretrained_agent/networks/eco/network_best_BA_200spin.pth"),
                    map_location="cpu", weights_only=True)
    out = {"ba200/" + k: v.detach().cpu().numpy().copy() for k, v in sd.items()}
    np.savez_compressed(os.path.join(HERE, "pretrained_ba200.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
