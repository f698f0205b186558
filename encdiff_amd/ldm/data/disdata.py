"""Shapes3D-style datasets (ldm/data/disdata.py:45-97, 749-775).

``Shapes3D`` reads an images array from an .npz (the reference reads 3dshapes.h5 with
h5py, which is not installed here); items are HWC float32 in [-1, 1] with an 'idx'
key, as the reference returns after ToTensor + Normalize(0.5, 0.5) + permute.
``SyntheticShapes3D`` produces the same item format from a seeded generator.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.utils.data import Dataset


class Shapes3D(Dataset):
    def __init__(self, path, key="images"):
        arr = np.load(path, mmap_mode="r")
        self.images = arr[key] if hasattr(arr, "files") else arr

    def __len__(self):
        return len(self.images)

    def __getitem__(self, i):
        img = torch.from_numpy(np.asarray(self.images[i], dtype=np.float32) / 127.5 - 1.0)
        return {"image": img, "idx": i}


class SyntheticShapes3D(Dataset):
    def __init__(self, n=480000, size=64, seed=0):
        self.n, self.size, self.seed = n, size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        return {"image": torch.rand(self.size, self.size, 3, generator=g) * 2 - 1, "idx": i}


class Shapes3DTrain(SyntheticShapes3D):
    """The reference's Shapes3DTrain binds a hard-coded /mnt path (disdata.py:749-775); here it
    is the synthetic stand-in of the same shape unless a ``path`` is given."""

    def __new__(cls, path=None, **kwargs):
        if path is not None:
            return Shapes3D(path)
        return super().__new__(cls)

    def __init__(self, path=None, **kwargs):
        super().__init__(**kwargs)
