"""Actor-critic policy of the reference, in PyTorch (the policy is not the hot
path; it stays in torch on the GPU).

Mirrors src/policies.py:
  * CustomExtractor (policies.py:21-113): one nn.Sequential per obs key built
    from the `arch` spec ([layer_name, params] lists, single.yaml:44-62); the
    first non-Embedding layer's input width is multiplied by n_frames_stack;
    mission -> Embedding -> GRU -> last hidden state; outputs concatenated in
    observation-space key order (direction 16 + image 64 + mission 128 = 208).
  * CustomPPOPolicy (policies.py:225-255) = SB3 ActorCriticPolicy with that
    extractor (shared by actor and critic), the SB3 default net_arch
    pi=[64,64] / vf=[64,64] with Tanh (CustomPPOPolicy pops and ignores
    `policy_kwargs`), orthogonal-init gains {extractor: sqrt 2, mlp: sqrt 2,
    action: 0.01, value: 1} applied through the reference's init_weights
    override (Conv2d: orthogonal(gain); Linear: N(0,1) rows normalised to unit
    norm, gain ignored), Adam(eps=optim_eps).
  * SB3 preprocess_obs: image /255 (normalize_images), other keys .float().

Engine-side addition (§8(f) rank 2, off by default): `mission_cache` runs the
mission GRU once per DISTINCT stacked mission row of a batch and gathers the
result.  The mission stack takes only (#missions x n_stack) values, so this
removes the dominant GRU cost at large N; gradients flow through the gather
(index backward = scatter-add), so training is the same computation up to
floating-point summation order.
"""
import math
import os

import numpy as np
import torch
from torch import nn

DEFAULT_ARCH = {
    "direction": [["Linear", [4, 16]]],
    "image": [["Conv2d", [3, 16, [2, 2]]], ["ReLU", []], ["MaxPool2d", [2]], ["Conv2d", [16, 32, [2, 2]]],
              ["ReLU", []], ["Conv2d", [32, 64, [2, 2]]], ["ReLU", []], ["Flatten", []]],
    "mission": [["Embedding", [32, 32]], ["GRU", [32, 128, 1, True, True]]],
}
OBS_KEYS = ("direction", "image", "mission")          # observation-space (Dict) key order


class Conv2dGemm(nn.Conv2d):
    """nn.Conv2d (same parameters, init and state_dict) that can compute as ONE GEMM
    over the whole batch: the kh*kw shifted views concatenated along channels (im2col
    without a per-sample loop) and contracted with the weight in a single matmul.
    Off by default (MGX_CONV_GEMM=1 enables it): MIOpen's own algorithms measured
    faster for the PPO update at minibatch 65,536.  Stride 1, no padding/dilation/
    groups (the reference's convs); anything else is plain nn.Conv2d."""

    enabled = os.environ.get("MGX_CONV_GEMM", "0") == "1"   # MIOpen measured faster at batch 64k

    def forward(self, x):
        if (not self.enabled or self.padding_mode != "zeros" or self.groups != 1 or tuple(self.stride) != (1, 1)
                or tuple(self.dilation) != (1, 1) or any(self.padding)):
            return super().forward(x)
        B, C, H, W = x.shape
        kh, kw = self.kernel_size
        oh, ow = H - kh + 1, W - kw + 1
        cols = torch.cat([x[:, :, dy:dy + oh, dx:dx + ow] for dy in range(kh) for dx in range(kw)], dim=1)
        cols = cols.permute(0, 2, 3, 1).reshape(B * oh * ow, kh * kw * C)           # [(b,y,x), (dy,dx,c)]
        wt = self.weight.permute(0, 2, 3, 1).reshape(self.out_channels, kh * kw * C)  # [out, (dy,dx,c)]
        out = torch.addmm(self.bias, cols, wt.t()) if self.bias is not None else cols @ wt.t()
        return out.reshape(B, oh, ow, self.out_channels).permute(0, 3, 1, 2)


def _pack_rows(tok):
    """Exact row key of a [B, L] token tensor (values < 32): 12 five-bit tokens per int64."""
    B, L = tok.shape
    pad = (-L) % 12
    if pad:
        tok = torch.nn.functional.pad(tok, (0, pad))
    t = tok.view(B, -1, 12).to(torch.int64)
    sh = torch.arange(12, device=tok.device, dtype=torch.int64) * 5
    return (t << sh).sum(-1)


class CustomExtractor(nn.Module):
    def __init__(self, obs_shapes, arch=None, n_frames_stack=4, mission_cache=False):
        super().__init__()
        arch = DEFAULT_ARCH if arch is None else arch
        self.n_frames_stack = n_frames_stack
        self.mission_cache = mission_cache
        # MIOpen's RNN rejects batches of 16,384 rows and more (miopenStatusBadParm, "Lengths must be
        # > 0"; 12,288 is accepted, with and without autograd: tools/gru_batch_probe.py on MI355X)
        self.gru_chunk = 8192
        self.aten_gru = os.environ.get("MGX_ATEN_GRU", "0") == "1"
        self.gru = False
        ext = {}
        total = 0
        for key in OBS_KEYS:
            if key not in arch:
                continue
            seq = nn.Sequential()
            for i, (name, params) in enumerate(arch[key]):
                cls = Conv2dGemm if name == "Conv2d" else getattr(nn, name)
                if params:
                    params = [list(p) if isinstance(p, (list, tuple)) else p for p in params]
                    if i == 0 and name != "Embedding":
                        params[0] = params[0] * n_frames_stack
                seq.add_module("%s_%s_%d" % (key, name, i), cls(*params) if params else cls())
                if name == "GRU":
                    self.gru = True
            ext[key] = seq
            total += self._out_width(seq, key, obs_shapes[key])
        self.extractors = nn.ModuleDict(ext)
        self.features_dim = total

    def _out_width(self, seq, key, shape):
        with torch.no_grad():
            if key == "mission":
                x = torch.zeros((1,) + tuple(shape), dtype=torch.int64)
                return self._mission(seq, x).shape[-1]
            return seq(torch.zeros((1,) + tuple(shape))).reshape(1, -1).shape[-1]

    def _mission(self, seq, tok):
        if self.gru:
            # aten_gru: ATen's per-step fused cell instead of MIOpen's RNN (measured slower
            # on MI355X at these shapes; kept as a switch)
            with torch.backends.cudnn.flags(enabled=not self.aten_gru):
                _, h = seq(tok)
            return h[-1]
        return seq(tok)

    def _mission_chunked(self, seq, tok):
        if tok.shape[0] <= self.gru_chunk:
            return self._mission(seq, tok)
        return torch.cat([self._mission(seq, c) for c in tok.split(self.gru_chunk)])

    def forward(self, obs):
        outs = []
        for key, seq in self.extractors.items():
            x = obs[key]
            if key == "mission":
                tok = x.to(torch.int64)
                if self.mission_cache:
                    keys = _pack_rows(tok)
                    uniq, inv = torch.unique(keys, dim=0, return_inverse=True)
                    u = uniq.shape[0]
                    # pad the distinct-row batch to a power of two: few distinct GRU shapes
                    # (MIOpen prepares one RNN plan per shape)
                    ub = max(64, 1 << (u - 1).bit_length())
                    first = torch.zeros(ub, dtype=torch.int64, device=tok.device)
                    first.scatter_(0, inv, torch.arange(tok.shape[0], device=tok.device))
                    out = self._mission_chunked(seq, tok.index_select(0, first)).index_select(0, inv)
                else:
                    out = self._mission_chunked(seq, tok)
            else:
                out = seq(x)
            if out.dim() > 2:
                out = out.reshape(out.shape[0], -1)
            outs.append(out)
        return torch.cat(outs, dim=1)


def _init_weights(module, gain=1.0):
    """CustomPPOPolicy.init_weights (policies.py:245-255)."""
    if isinstance(module, nn.Conv2d):                  # (Conv2dGemm is an nn.Conv2d)
        nn.init.orthogonal_(module.weight, gain=gain)
        if module.bias is not None:
            module.bias.data.fill_(0.0)
    if isinstance(module, nn.Linear):
        module.weight.data.normal_(0, 1)
        module.weight.data *= 1 / torch.sqrt(module.weight.data.pow(2).sum(1, keepdim=True))
        if module.bias is not None:
            module.bias.data.fill_(0)


def preprocess(obs):
    """SB3 preprocess_obs for the Dict space: image /255, the rest float.  Float inputs are taken
    as already preprocessed (mgx_gather's f32 output is exactly this, computed in the gather)."""
    img = obs["image"]
    return {"image": img if img.is_floating_point() else img.float() / 255.0,
            "direction": obs["direction"].float(), "mission": obs["mission"]}


class ActorCriticPolicy(nn.Module):
    def __init__(self, n_stack=4, arch=None, n_actions=7, net_arch=None, optim_eps=1e-8, lr=3e-4,
                 mission_cache=False):
        super().__init__()
        shapes = {"direction": (4 * n_stack,), "image": (3 * n_stack, 7, 7), "mission": (32 * n_stack,)}
        self.features_extractor = CustomExtractor(shapes, arch, n_stack, mission_cache)
        net_arch = net_arch or {"pi": [64, 64], "vf": [64, 64]}
        fd = self.features_extractor.features_dim

        def mlp(widths):
            layers, w = [], fd
            for h in widths:
                layers += [nn.Linear(w, h), nn.Tanh()]
                w = h
            return nn.Sequential(*layers), w

        self.policy_net, dpi = mlp(net_arch["pi"])
        self.value_net_body, dvf = mlp(net_arch["vf"])
        self.action_net = nn.Linear(dpi, n_actions)
        self.value_net = nn.Linear(dvf, 1)
        for mod, gain in ((self.features_extractor, math.sqrt(2)), (self.policy_net, math.sqrt(2)),
                          (self.value_net_body, math.sqrt(2)), (self.action_net, 0.01), (self.value_net, 1.0)):
            mod.apply(lambda m, g=gain: _init_weights(m, g))
        self.optimizer = torch.optim.Adam(self.parameters(), lr=lr, eps=optim_eps)

    def _latent(self, obs):
        f = self.features_extractor(preprocess(obs))
        return self.policy_net(f), self.value_net_body(f)

    def forward(self, obs, deterministic=False):
        """-> actions [B] int64, values [B], log_prob [B] (SB3 ActorCriticPolicy.forward)."""
        pi, vf = self._latent(obs)
        dist = torch.distributions.Categorical(logits=self.action_net(pi))
        actions = dist.probs.argmax(1) if deterministic else dist.sample()
        return actions, self.value_net(vf).flatten(), dist.log_prob(actions)

    @torch.no_grad()
    def predict(self, obs, deterministic=False):
        """SB3 BasePolicy.predict (actions only): mode of the action distribution
        (argmax of its probs) when deterministic, else a sample."""
        return self.forward(obs, deterministic)[0]

    def evaluate_actions(self, obs, actions):
        pi, vf = self._latent(obs)
        dist = torch.distributions.Categorical(logits=self.action_net(pi))
        return self.value_net(vf).flatten(), dist.log_prob(actions), dist.entropy()

    def predict_values(self, obs):
        _, vf = self._latent(obs)
        return self.value_net(vf).flatten()


def n_params(module):
    return int(sum(np.prod(p.shape) for p in module.parameters()))
