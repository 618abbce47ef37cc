"""Tiny CPU classifier used only by the CPU plumbing tests of the training loop (config -> DataModule
-> LitClassifier -> Trainer).  The product models (EnvNetV2, ASTModel) run only on the HIP path."""
import torch
import torch.nn as nn


class TinyNet(nn.Module):
    def __init__(self, num_classes: int = 50, in_samples: int = 64):
        super().__init__()
        self.net = nn.Sequential(nn.Flatten(), nn.Linear(in_samples, 32), nn.ReLU(), nn.Linear(32, num_classes))
        self.bn = nn.BatchNorm1d(32)  # a buffer-carrying module for the DDP buffer broadcast test

    def forward(self, x):
        return self.net(x)


class _EmitFn(torch.autograd.Function):
    """Linear -> ReLU -> Linear as ONE autograd node whose backward hands the head's gradients to the
    data-parallel reducer through ``model._grad_ready`` (and fc1's weight gradient as two row chunks
    through ``model._grad_chunk_ready``) and returns None for them — the contract of the EnvNetV2 /
    AST autograd nodes (envnet_hip.py emit() and its FC1 chunks, ast_hip.py)."""

    @staticmethod
    def forward(ctx, model, x, w1, b1, w2, b2):
        h = torch.relu(x @ w1.t() + b1)
        ctx.save_for_backward(x, h, w1, w2)
        ctx.model = model
        return h @ w2.t() + b2

    @staticmethod
    def backward(ctx, g):
        x, h, w1, w2 = ctx.saved_tensors
        gw2, gb2 = g.t() @ h, g.sum(0)
        dh = (g @ w2) * (h > 0)
        gw1, gb1 = dh.t() @ x, dh.sum(0)
        ready = getattr(ctx.model, "_grad_ready", None)
        if ready is not None:
            ready([(ctx.model.fc2.weight, gw2), (ctx.model.fc2.bias, gb2)])
            gw2 = gb2 = None
        chunk = getattr(ctx.model, "_grad_chunk_ready", None)
        if chunk is not None:  # fc1.weight in two row chunks (the EnvNet FC1 path, envnet_hip.py)
            gw1 = gw1.contiguous()
            chunk(ctx.model.fc1.weight, gw1, gw1[:16], False)
            chunk(ctx.model.fc1.weight, gw1, gw1[16:], True)
            gw1 = None
        return None, None, gw1, gb1, gw2, gb2


class EmitNet(nn.Module):
    def __init__(self, num_classes: int = 5, in_samples: int = 16):
        super().__init__()
        self.fc1 = nn.Linear(in_samples, 32)
        self.fc2 = nn.Linear(32, num_classes)
        self.bn = nn.BatchNorm1d(4)

    def forward(self, x):
        x = x.reshape(x.shape[0], -1)
        return _EmitFn.apply(self, x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias)
