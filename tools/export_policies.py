"""Convert the shipped evaluation policies (Simulation/AGENT_NNS/<cfg>/<cfg>_
checkpoint_actor / _checkpoint_encoder, loaded with weights_only=True) into one
safetensors file per tremor configuration under policies/ (git-ignored), for
tools/eval_policies.py on the GPU box, where /root/reference does not exist.
Only what evaluation reads is kept: the checkpoint actor and the checkpoint
encoder's zs layers (Evaluate_control_performance.py:126 -> select_action with
use_checkpoint=True, TD7_multi_agent_Pink_noise.py:212-214).

usage: python tools/export_policies.py [--src /root/reference/Simulation/AGENT_NNS]
"""
import argparse
import os

import torch
from safetensors.torch import save_file

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="/root/reference/Simulation/AGENT_NNS")
    ap.add_argument("--out", default=os.path.join(REPO, "policies"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for cfg in sorted(os.listdir(a.src)):
        base = os.path.join(a.src, cfg, cfg)
        actor = torch.load(base + "_checkpoint_actor", map_location="cpu", weights_only=True)
        enc = torch.load(base + "_checkpoint_encoder", map_location="cpu", weights_only=True)
        t = {f"actor.{k}": v.float().contiguous() for k, v in actor.items()}
        t.update({f"encoder.{k}": v.float().contiguous() for k, v in enc.items() if k.split(".")[0] in ("zs1", "zs2", "zs3")})
        save_file(t, os.path.join(a.out, cfg + ".safetensors"))
        print(cfg, sum(v.numel() for v in t.values()), "parameters")


if __name__ == "__main__":
    main()
