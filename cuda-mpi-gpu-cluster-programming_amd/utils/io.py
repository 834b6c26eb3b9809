"""Weight checkpoints (the reference has none; runs used constant/random weights).

* ``save_weights`` / ``load_weights``: safetensors files (loading executes nothing from the file).
* ``save_weights_raw`` / ``load_weights_raw``: a directory of little-endian fp32 blobs
  (``w1.bin b1.bin w2.bin b2.bin`` + ``shapes.json``) — the format the native CLI reads with
  ``anx --weights DIR``.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch
from safetensors.torch import load_file, save_file


def save_weights(path: str, weights: dict) -> None:
    save_file({k: v.detach().to("cpu", torch.float32).contiguous() for k, v in weights.items()}, path)


def load_weights(path: str) -> dict:
    return load_file(path)


def save_weights_raw(directory: str, weights: dict) -> None:
    os.makedirs(directory, exist_ok=True)
    shapes = {}
    for k, v in weights.items():
        a = v.detach().to("cpu", torch.float32).contiguous().numpy()
        a.astype("<f4").tofile(os.path.join(directory, f"{k}.bin"))
        shapes[k] = list(a.shape)
    with open(os.path.join(directory, "shapes.json"), "w") as f:
        json.dump(shapes, f)


def load_weights_raw(directory: str) -> dict:
    with open(os.path.join(directory, "shapes.json")) as f:
        shapes = json.load(f)
    return {k: torch.from_numpy(np.fromfile(os.path.join(directory, f"{k}.bin"), dtype="<f4").reshape(s))
            for k, s in shapes.items()}
