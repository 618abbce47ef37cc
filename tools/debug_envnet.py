"""Debug: compare EnvNet HIP intermediates with torch (CPU f64) layer by layer."""
import sys
sys.path[:0] = [".", "dl-sound-classification_amd"]
import numpy as np
import torch
import torch.nn.functional as F
from oracle.synth import synth_waveform
from oracle import envnet as oenv
from tests._util import envnet_with_hash_params

dev = torch.device("cuda:0")
x = torch.from_numpy(synth_waveform(21, 2, 220_500)[:, None, :])
params = oenv.to_torch(oenv.hash_params(100))
pd = {k: v.double() for k, v in params.items()}

def rel(a, b):
    a = a.double().cpu(); b = b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))

for mode in ("eval", "train", "eval"):
    m = envnet_with_hash_params(dev)
    m.train(mode == "train")
    m._debug_capture = True
    with torch.no_grad():
        z = m(x.to(dev))
    s = m._debug
    tr = mode == "train"
    # reference intermediates
    h = x.double().unsqueeze(2)
    y1 = F.conv2d(h, pd["frontend.0.weight"], pd["frontend.0.bias"], stride=(1, 2))
    print(mode, "y1", rel(s["y1"].view(2, -1, 32).permute(0, 2, 1), y1[:, :, 0]))
    def bn(y, name):
        if tr:
            mu = y.mean(dim=(0, 2, 3)); var = y.var(dim=(0, 2, 3), unbiased=False)
        else:
            mu = pd[name + ".running_mean"]; var = pd[name + ".running_var"]
        return F.relu((y - mu[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + 1e-5) * pd[name + ".weight"][None, :, None, None] + pd[name + ".bias"][None, :, None, None])
    a1 = bn(y1, "frontend.1")
    print(mode, "bn1 mean", rel(s["bn1"].mean, a1.new_tensor(y1.mean(dim=(0,2,3)).numpy()) if tr else pd["frontend.1.running_mean"]))
    y2 = F.conv2d(a1, pd["frontend.3.weight"], pd["frontend.3.bias"], stride=(1, 2))
    print(mode, "y2", rel(s["y2"].view(2, -1, 64).permute(0, 2, 1), y2[:, :, 0]))
    a2 = bn(y2, "frontend.4")
    p0 = F.max_pool2d(a2, (1, 64), (1, 64)).transpose(1, 2)
    print(mode, "X0", rel(s["X0"], p0[:, 0]))
    hh = p0
    for blk in range(4):
        ts = s["trunk"][blk]
        ya = F.conv2d(hh, pd[f"trunk.{blk}.0.weight"], pd[f"trunk.{blk}.0.bias"])
        print(mode, blk, "ya", rel(ts["ya"].view(ya.shape[0], ya.shape[2], ya.shape[3], -1).permute(0, 3, 1, 2), ya))
        aa = bn(ya, f"trunk.{blk}.1")
        yb = F.conv2d(aa, pd[f"trunk.{blk}.3.weight"], pd[f"trunk.{blk}.3.bias"])
        print(mode, blk, "yb", rel(ts["yb"].view(yb.shape[0], yb.shape[2], yb.shape[3], -1).permute(0, 3, 1, 2), yb))
        ab = bn(yb, f"trunk.{blk}.4")
        k = oenv.POOLS[f"trunk.{blk}"]
        hh = F.max_pool2d(ab, k[0], k[1])
    print(mode, "flat", rel(s["flat"], hh.flatten(1)))
    h1 = F.relu(F.linear(hh.flatten(1), pd["classifier.1.weight"], pd["classifier.1.bias"]))
    print(mode, "h1", rel(s["h1"], h1))
    h2 = F.relu(F.linear(h1, pd["classifier.4.weight"], pd["classifier.4.bias"]))
    print(mode, "h2", rel(s["h2"], h2))
    zz = F.linear(h2, pd["classifier.7.weight"], pd["classifier.7.bias"])
    print(mode, "logits", rel(z, zz))
