"""torch modules with the reference's parameter names, registration order and
initialisation, whose parameters are VIEWS into the flat device vector the
HIP kernels read and update.

They exist so that `FBSNN.model` behaves like the reference attribute
(state_dict / load_state_dict / parameters / torch.save checkpoints,
nd_BSPDE_case.py:445-456).  Training, prediction and net_u never call their
forward(); it is kept for callers that differentiate the network directly
(e.g. the reference's StabilityCheck), which is outside the hot path.

Layouts (state_dict order):
  FC        DeepBSDE.py:166-172         0.weight, 0.bias, 2.weight, ...
  NAIS-Net  DeepBSDE.py:23-65           input_layer, hidden_layers.k, output_layer, input_layers.k
  Resnet    DeepBSDE.py:23-65 (stable=False)
  Naisnet   Functions/naisnet.py:6-96   layer1, layer2, layer2_input, layer3, ...
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class Sine(nn.Module):
    """Functions/Sine.py:6-12."""

    def forward(self, x):
        return torch.sin(x)


def activation_module(name):
    table = {"Sine": Sine, "ReLU": nn.ReLU, "Tanh": nn.Tanh}
    if name not in table:
        raise ValueError(f"activation {name!r} is not one of {sorted(table)}")
    return table[name]()


def _neg_projected(lin, eps=0.01):
    # Functions/naisnet.py:30-39; returns -A for F.linear
    rtr = lin.weight.t() @ lin.weight
    n = torch.norm(rtr)
    if n > 1 - 2 * eps:
        rtr = (1 - 2 * eps) ** 0.5 * rtr / n ** 0.5
    return -(rtr + eps * torch.eye(rtr.shape[0], device=rtr.device, dtype=rtr.dtype))


class Resnet(nn.Module):
    def __init__(self, layers, stable, activation):
        super().__init__()
        self.stable = stable
        self.activation_function = activation
        self.input_layer = nn.Linear(layers[0], layers[1])
        self.hidden_layers = nn.ModuleList(nn.Linear(layers[i], layers[i + 1]) for i in range(1, len(layers) - 2))
        self.output_layer = nn.Linear(layers[-2], layers[-1])
        if stable:
            self.input_layers = nn.ModuleList(nn.Linear(layers[0], layers[i]) for i in range(1, len(layers) - 1))

    def forward(self, x):
        h = self.activation_function(self.input_layer(x))
        for k, lin in enumerate(self.hidden_layers):
            a = F.linear(h, _neg_projected(lin), lin.bias) + self.input_layers[k](x) if self.stable else lin(h)
            h = self.activation_function(a) + h
        return self.output_layer(h)


class Naisnet(nn.Module):
    def __init__(self, layers, activation):
        super().__init__()
        n = len(layers)
        if n not in (4, 5, 6):
            raise ValueError("Naisnet supports len(layers) in {4, 5, 6}")
        self.layers = list(layers)
        self.activation = activation
        self.layer1 = nn.Linear(layers[0], layers[1])
        self.layer2 = nn.Linear(layers[1], layers[2])
        self.layer2_input = nn.Linear(layers[0], layers[2])
        self.layer3 = nn.Linear(layers[2], layers[3])
        if n >= 5:
            self.layer3_input = nn.Linear(layers[0], layers[3])
            self.layer4 = nn.Linear(layers[3], layers[4])
        if n == 6:
            self.layer4_input = nn.Linear(layers[0], layers[4])
            self.layer5 = nn.Linear(layers[4], layers[5])

    def forward(self, x):
        n = len(self.layers)
        h = self.activation(self.layer1(x))
        for k in range(2, n - 1):
            lin, inj = getattr(self, f"layer{k}"), getattr(self, f"layer{k}_input")
            h = self.activation(F.linear(h, _neg_projected(lin), lin.bias) + inj(x)) + h
        return getattr(self, f"layer{n - 1}")(h)


def make_model(mode, layers, activation):
    """Build on the CPU with the reference's init (nn.Linear default, then
    xavier_uniform_ on every weight in apply() order, DeepBSDE.py:180-187), so a
    given torch.manual_seed yields the reference's CPU-run weights."""
    act = activation_module(activation)
    if mode == "FC":
        mods = []
        for i in range(len(layers) - 2):
            mods += [nn.Linear(layers[i], layers[i + 1]), act]
        mods.append(nn.Linear(layers[-2], layers[-1]))
        model = nn.Sequential(*mods)
    elif mode in ("NAIS-Net", "Resnet"):
        model = Resnet(layers, mode == "NAIS-Net", act)
    elif mode == "Naisnet":
        model = Naisnet(layers, act)
    else:
        raise ValueError(f"mode {mode!r} is not one of ['FC', 'NAIS-Net', 'Naisnet', 'Resnet']")
    model.apply(lambda m: torch.nn.init.xavier_uniform_(m.weight) if isinstance(m, nn.Linear) else None)
    return model


def make_heston_model(mode, layers, activation, n_in):
    """heston_dnnpde.py:519-585: the base FBSNN builds the network on the
    reference's `layers` (input D + 1) with the usual init, HestonFBSNN then
    replaces every input-facing Linear by one with n_in = 1 + 2k inputs
    (t, S_1..S_k, v_1..v_k) and re-initialises all parameters (xavier_uniform_
    gain 0.5 on matrices, zeros on vectors), in that RNG order."""
    model = make_model(mode, layers, activation)
    if mode == "FC":
        model[0] = nn.Linear(n_in, layers[1])
    elif mode == "Naisnet":
        model.layer1 = nn.Linear(n_in, layers[1])
        model.layer2_input = nn.Linear(n_in, layers[2])
        if len(layers) >= 5:
            model.layer3_input = nn.Linear(n_in, layers[3])
        if len(layers) == 6:
            model.layer4_input = nn.Linear(n_in, layers[4])
    else:
        raise ValueError("HestonFBSNN supports the 'FC' and 'Naisnet' modes (heston_dnnpde.py:156-167)")
    for prm in model.parameters():
        if prm.dim() > 1:
            torch.nn.init.xavier_uniform_(prm, gain=0.5)
        else:
            torch.nn.init.zeros_(prm)
    return model


def flatten_into(model, device):
    """Copy the model's state into one flat fp32 device vector and rebind every
    parameter as a view of it.  Returns the flat vector."""
    sd = model.state_dict()
    flat = torch.cat([p.detach().reshape(-1).float() for p in sd.values()]).to(device)
    bind(model, flat)
    return flat


def bind(model, flat):
    off = 0
    params = dict(model.named_parameters())
    for name, p in model.state_dict().items():
        n = p.numel()
        params[name].data = flat[off:off + n].view(p.shape)
        off += n
    if off != flat.numel():
        raise ValueError("flat parameter vector does not match the model layout")
