"""Drop-in ``utility_layers`` module (utility_layers.py of the reference):
StochasticDepth and the SdPModel base class (config / IO surface the harnesses
use: from_dict, return_num_params, save_model, from_pretrained, layer_test).

TecherModel (torch.hub teacher wrapper, utility_layers.py:62-76) is out of scope
(remote fetch, never on the forward path) and not provided.
"""
from __future__ import annotations

from typing import Union

import torch
from torch import nn as nn


class StochasticDepth(torch.nn.Module):
    """Per-sample drop path (utility_layers.py:7-27): identity in eval mode,
    Bernoulli(1-p)/(1-p) scaling per sample in training mode."""

    def __init__(self, p: float = 0.2):
        super().__init__()
        assert 0 < p < 1, "p must be a positive number or <1"
        self.p = p

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            size = (x.shape[0],) + (1,) * (x.ndim - 1)
            noise_x = torch.empty(size, dtype=x.dtype, device=x.device, requires_grad=False).bernoulli(1 - self.p).div(1 - self.p)
            return noise_x * x
        return x


class SdPModel(nn.Module):
    """Base class with the reference's utility surface (utility_layers.py:93-198)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.config = {}

    def layer_init(self):
        pass

    def layer_test(self, input=None, output=None, loss_fn=None):
        """Forward-hook mean/std probe (utility_layers.py:104-151).  Hooks fire on
        the modules the HIP forward actually invokes (the model switches to its
        module-by-module path while hooks are attached).  The default probe input
        is created on the model's device (the reference creates it on the CPU)."""
        means, stds, norms = [], [], []
        self.eval()

        @torch.no_grad()
        def forward_hook(module, inp, out):
            if isinstance(out, Union[tuple, list]):
                for o in out:
                    means.append(o.float().mean().item())
                    stds.append(o.float().std().item())
            else:
                means.append(out.float().mean().item())
                stds.append(out.float().std().item())

        handles = [m.register_forward_hook(forward_hook) for m in self.modules()]
        try:
            if not input:
                dev = next(self.parameters()).device
                self(torch.randn(1, 3, 224, 224, device=dev))
            else:
                self(input)
        finally:
            for h in handles:
                h.remove()
        self.train()
        return {"forward_means": means, "Forward_std": stds, "Backward_norm": norms}

    def return_num_params(self) -> dict:
        params = sum([param.numel() * 1j if param.requires_grad else param.numel() for param in self.parameters()])
        return {"Trainable_params": int(params.imag), "Non_trainable_params": int(params.real)}

    @classmethod
    def from_dict(cls, **kwargs):
        model = cls(**kwargs)
        model.config = kwargs
        return model

    @classmethod
    def from_pretrained(cls, file_name):
        try:
            dict_ = torch.load(file_name, weights_only=True, map_location="cpu")
            config = dict_["config"]
            state_dict = dict_["state_dict"]
            model = cls.from_dict(**config)
            model.load_state_dict(state_dict)
            print(f"Model loaded successfully!!!! The current configuration is {config}")
        except Exception as e:
            print(f"Something went wrong with {e}")
        return model

    def save_model(self, file_name=None):
        fn = "Model" if file_name is None else file_name
        model = {"state_dict": self.state_dict(), "config": self.config}
        try:
            torch.save(model, f"{fn}.pt")
            print(f"Model saved succesfully, see the file {fn}.pt for the weights and config file!!!")
        except Exception as exp:
            print(f"Something went wrong with {exp}!!!!!")
