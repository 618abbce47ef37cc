"""Tiny CPU classifier used only by the CPU plumbing tests of the training loop (config -> DataModule
-> LitClassifier -> Trainer).  The product models (EnvNetV2, ASTModel) run only on the HIP path."""
import torch.nn as nn


class TinyNet(nn.Module):
    def __init__(self, num_classes: int = 50, in_samples: int = 64):
        super().__init__()
        self.net = nn.Sequential(nn.Flatten(), nn.Linear(in_samples, 32), nn.ReLU(), nn.Linear(32, num_classes))
        self.bn = nn.BatchNorm1d(32)  # a buffer-carrying module for the DDP buffer broadcast test

    def forward(self, x):
        return self.net(x)
