"""Mirror of the data plumbing the configs target (``main.DataModuleFromConfig``,
main_val.py:214-318) -- host-side, outside the HIP hot path."""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, Dataset

from encdiff_amd.ldm.util import instantiate_from_config


class WrappedDataset(Dataset):
    def __init__(self, dataset):
        self.data = dataset

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self.data[idx]


class DataModuleFromConfig:
    """main_val.py:243-318 without Lightning: instantiate the dataset configs and hand out
    torch DataLoaders with the configured batch size / workers."""

    def __init__(self, batch_size, train=None, validation=None, test=None, predict=None, wrap=False,
                 num_workers=None, shuffle_test_loader=False, use_worker_init_fn=False, shuffle_val_dataloader=False):
        self.batch_size = batch_size
        self.num_workers = num_workers if num_workers is not None else batch_size * 2
        self.dataset_configs = {k: v for k, v in dict(train=train, validation=validation, test=test,
                                                      predict=predict).items() if v is not None}
        self.wrap = wrap
        self.datasets = {}

    def setup(self, stage=None):
        self.datasets = {k: instantiate_from_config(c) for k, c in self.dataset_configs.items()}
        if self.wrap:
            self.datasets = {k: WrappedDataset(d) for k, d in self.datasets.items()}

    def train_dataloader(self):
        return DataLoader(self.datasets["train"], batch_size=self.batch_size, num_workers=self.num_workers,
                          shuffle=True, drop_last=True)

    def val_dataloader(self):
        return DataLoader(self.datasets["validation"], batch_size=self.batch_size, num_workers=self.num_workers)
