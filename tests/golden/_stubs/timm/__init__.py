"""Offline restatement of the timm 1.0.16 VisionTransformer surface the reference's
ASTModel uses (uv.lock:2136): create_model(...) -> object with embed_dim, pos_embed,
patch_embed.proj, cls_token, blocks (Block: LN eps 1e-6 -> qkv(bias) -> SDPA -> proj;
LN -> fc1 -> GELU -> fc2) and norm. Weights are synthetic (pretrained DeiT weights need
the network). Used ONLY by tests/golden/make_golden.py."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        B, N, C = x.shape
        qkv = self.qkv(x).reshape(B, N, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        x = F.scaled_dot_product_attention(q, k, v, dropout_p=0.0)
        x = x.transpose(1, 2).reshape(B, N, C)
        return self.proj(x)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class _PatchEmbed(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.proj = nn.Conv2d(3, dim, kernel_size=16, stride=16)


class VisionTransformer(nn.Module):
    def __init__(self, embed_dim=768, depth=12, num_heads=12, grid=24):
        super().__init__()
        self.embed_dim = embed_dim
        self.patch_embed = _PatchEmbed(embed_dim)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, grid * grid + 1, embed_dim))
        self.blocks = nn.Sequential(*[Block(embed_dim, num_heads) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)


# Synthetic weights are injected by the golden script through this hook.
STATE_HOOK = None


def create_model(name, pretrained=False, **kw):
    assert name == "deit_base_patch16_384", name
    m = VisionTransformer()
    if STATE_HOOK is not None:
        sd = STATE_HOOK()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return m
