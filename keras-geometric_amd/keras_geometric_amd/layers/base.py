"""Keras-style layer scaffolding on torch.nn.Module.

The reference layers subclass `keras.layers.Layer` (Keras 3, torch backend).
Keras is not installed in this environment, so the drop-in
layers here reproduce the parts of the Keras Layer contract the reference and
its tests use — `layer([x, edge_index], training=None)`, lazy `build()` on the
first call, `add_weight`, `get_weights`/`set_weights`, `get_config`/
`from_config`, `compute_dtype` — on a `torch.nn.Module`, with parameters living
on the ROCm device of the inputs.  INTEGRATION.md shows the Keras-side binding.
"""

from __future__ import annotations

import math
from typing import Any, Callable

import numpy as np
import torch

_GLOBAL_SEED: int | None = None


def set_random_seed(seed: int) -> None:
    """Seed weight initialisation (keras.utils.set_random_seed analogue)."""
    global _GLOBAL_SEED
    _GLOBAL_SEED = int(seed)
    torch.manual_seed(seed)


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError(
            "keras_geometric_amd runs on MI355X (ROCm) GPUs only and no GPU is visible; "
            "there is no CPU execution path."
        )
    return torch.device("cuda", torch.cuda.current_device())


def to_device_tensor(x, dtype: torch.dtype, device: torch.device | None = None) -> torch.Tensor:
    """numpy / list / tensor -> tensor of `dtype` on the kgx device."""
    if isinstance(x, torch.Tensor):
        dev = x.device if x.device.type == "cuda" else (device or default_device())
        return x.to(device=dev, dtype=dtype)
    arr = np.asarray(x)
    return torch.as_tensor(arr).to(device=device or default_device(), dtype=dtype)


def shape_of(x) -> tuple:
    return tuple(x.shape) if hasattr(x, "shape") else tuple(np.asarray(x).shape)


# ---------------------------------------------------------------------------
# initializers (Keras names)
# ---------------------------------------------------------------------------
class Constant:
    def __init__(self, value: float = 0.0):
        self.value = float(value)

    def __call__(self, shape, device):
        return torch.full(shape, self.value, dtype=torch.float32, device=device)

    def get_config(self):
        return {"value": self.value}


def _fans(shape) -> tuple[int, int]:
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    receptive = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    return shape[-2] * receptive, shape[-1] * receptive


def get_initializer(spec) -> Callable:
    if callable(spec) and not isinstance(spec, str):
        return spec
    name = (spec or "zeros").lower() if isinstance(spec, str) else "zeros"

    def glorot_uniform(shape, device):
        fan_in, fan_out = _fans(shape)
        limit = math.sqrt(6.0 / max(1, fan_in + fan_out))
        return (torch.rand(shape, device=device) * 2 - 1) * limit

    def glorot_normal(shape, device):
        fan_in, fan_out = _fans(shape)
        std = math.sqrt(2.0 / max(1, fan_in + fan_out))
        return torch.nn.init.trunc_normal_(torch.empty(shape, device=device), std=std, a=-2 * std, b=2 * std)

    def he_uniform(shape, device):
        fan_in, _ = _fans(shape)
        limit = math.sqrt(6.0 / max(1, fan_in))
        return (torch.rand(shape, device=device) * 2 - 1) * limit

    def he_normal(shape, device):
        fan_in, _ = _fans(shape)
        std = math.sqrt(2.0 / max(1, fan_in))
        return torch.nn.init.trunc_normal_(torch.empty(shape, device=device), std=std, a=-2 * std, b=2 * std)

    table = {
        "glorot_uniform": glorot_uniform,
        "glorot_normal": glorot_normal,
        "he_uniform": he_uniform,
        "he_normal": he_normal,
        "zeros": lambda shape, device: torch.zeros(shape, device=device),
        "ones": lambda shape, device: torch.ones(shape, device=device),
    }
    if name not in table:
        raise ValueError(f"Unknown initializer: {spec}")
    fn = table[name]
    fn.__name__ = name
    return fn


def serialize_initializer(init) -> Any:
    return getattr(init, "__name__", None) or (
        {"class_name": type(init).__name__, "config": init.get_config()} if hasattr(init, "get_config") else str(init)
    )


# ---------------------------------------------------------------------------
# activations (Keras names)
# ---------------------------------------------------------------------------
_ACTIVATIONS: dict[str, Callable[[torch.Tensor], torch.Tensor]] = {
    "relu": torch.relu,
    "linear": lambda x: x,
    "sigmoid": torch.sigmoid,
    "tanh": torch.tanh,
    "elu": torch.nn.functional.elu,
    "gelu": lambda x: torch.nn.functional.gelu(x, approximate="none"),
    "leaky_relu": lambda x: torch.nn.functional.leaky_relu(x, 0.2),
    "softmax": lambda x: torch.softmax(x, dim=-1),
}


def get_activation(spec):
    if spec is None:
        return None
    if callable(spec):
        return spec
    if spec not in _ACTIVATIONS:
        raise ValueError(f"Unknown activation: {spec}")
    fn = _ACTIVATIONS[spec]
    try:
        fn.__name__ = spec
    except (AttributeError, TypeError):
        pass
    return fn


def serialize_activation(fn) -> str | None:
    if fn is None:
        return None
    for k, v in _ACTIVATIONS.items():
        if v is fn:
            return k
    return getattr(fn, "__name__", str(fn))


# ---------------------------------------------------------------------------
# Layer
# ---------------------------------------------------------------------------
class Layer(torch.nn.Module):
    """Minimal Keras-3 Layer contract on torch.nn.Module."""

    def __init__(self, name: str | None = None, dtype: str | None = None, trainable: bool = True, **kwargs):
        super().__init__()
        if kwargs:
            raise TypeError(f"Unrecognized keyword arguments passed to {type(self).__name__}: {kwargs}")
        self.name = name or type(self).__name__.lower()
        self.dtype_policy = dtype or "float32"
        self.compute_dtype = "float32"
        self.dtype = "float32"
        self.trainable = trainable
        self.built = False
        self._weight_order: list[str] = []

    # -- Keras API ---------------------------------------------------------
    def build(self, input_shape) -> None:
        self.built = True

    def call(self, *args, **kwargs):
        raise NotImplementedError

    def forward(self, inputs, *args, **kwargs):
        if not self.built:
            shapes = [shape_of(t) if t is not None else None for t in inputs] if isinstance(
                inputs, (list, tuple)
            ) else shape_of(inputs)
            self._build_device = _first_device(inputs)
            self.build(shapes)
            self.built = True
        return self.call(inputs, *args, **kwargs)

    def add_weight(self, shape, initializer="glorot_uniform", name: str = "weight", trainable: bool = True,
                   **_ignored) -> torch.nn.Parameter:
        dev = getattr(self, "_build_device", None) or default_device()
        init = get_initializer(initializer) if not isinstance(initializer, Constant) else initializer
        p = torch.nn.Parameter(init(tuple(int(s) for s in shape), dev).float(), requires_grad=trainable)
        attr = name
        i = 1
        while attr in self._parameters:
            attr = f"{name}_{i}"
            i += 1
        if attr in self.__dict__:  # placeholder attribute (e.g. self.kernel = None in __init__)
            del self.__dict__[attr]
        self.register_parameter(attr, p)
        self._weight_order.append(attr)
        return p

    @property
    def weights(self) -> list[torch.nn.Parameter]:
        """Own weights in creation order, then sub-layers' (Keras Layer.weights order)."""
        out = [self._parameters[k] for k in self._weight_order]

        def visit(mod):
            for m in mod.children():
                if isinstance(m, Layer):
                    out.extend(m.weights)
                else:  # containers such as ModuleList
                    visit(m)

        visit(self)
        return out

    def get_weights(self) -> list[np.ndarray]:
        return [w.detach().cpu().numpy() for w in self.weights]

    def set_weights(self, weights) -> None:
        mine = self.weights
        if len(weights) != len(mine):
            raise ValueError(f"set_weights: expected {len(mine)} arrays, got {len(weights)}")
        with torch.no_grad():
            for p, v in zip(mine, weights):
                t = torch.as_tensor(np.asarray(v), dtype=torch.float32)
                if tuple(t.shape) != tuple(p.shape):
                    raise ValueError(f"set_weights: shape {tuple(t.shape)} vs {tuple(p.shape)}")
                p.copy_(t.to(p.device))

    def get_config(self) -> dict[str, Any]:
        return {"name": self.name, "trainable": self.trainable, "dtype": self.dtype_policy}

    @classmethod
    def from_config(cls, config: dict[str, Any]):
        return cls(**config)


def _first_device(inputs) -> torch.device | None:
    items = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    for t in items:
        if isinstance(t, torch.Tensor) and t.device.type == "cuda":
            return t.device
        if isinstance(t, (list, tuple)):
            d = _first_device(t)
            if d is not None:
                return d
    return None


class Dense(Layer):
    """keras.layers.Dense: activation(x @ kernel + bias) (GEMM on hipBLASLt/MFMA)."""

    def __init__(self, units: int, activation=None, use_bias: bool = True,
                 kernel_initializer="glorot_uniform", bias_initializer="zeros", **kwargs):
        for k in ("kernel_regularizer", "bias_regularizer", "kernel_constraint", "bias_constraint"):
            kwargs.pop(k, None)
        super().__init__(**kwargs)
        self.units = int(units)
        self.activation = get_activation(activation)
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer
        self.kernel = None
        self.bias = None

    def build(self, input_shape) -> None:
        in_dim = int(input_shape[-1])
        self.kernel = self.add_weight((in_dim, self.units), self.kernel_initializer, name="kernel")
        if self.use_bias:
            self.bias = self.add_weight((self.units,), self.bias_initializer, name="bias")
        self.built = True

    def forward(self, x, *args, **kwargs):
        if not self.built:
            self._build_device = x.device if isinstance(x, torch.Tensor) else None
            self.build(shape_of(x))
        return self.call(x)

    def call(self, x):
        if x.dim() == 2 and x.is_cuda:
            from .. import ops as kops  # deferred: ops imports the layers' graph cache

            if kops.dense_supported(x, self.kernel):
                # kgx_dense: bias and ReLU in the MFMA kernel's epilogue (differentiable)
                relu = self.activation is torch.relu
                y = kops.dense(x, self.kernel, self.bias if self.use_bias else None, relu=relu)
                return y if (relu or self.activation is None) else self.activation(y)
        if self.use_bias and x.dim() == 2:
            if self.activation is torch.relu and x.is_cuda and not torch.is_grad_enabled():
                # inference: bias + ReLU in the GEMM epilogue (one pass over the output;
                # this fused op has no autograd formula)
                return torch._addmm_activation(self.bias, x, self.kernel)
            y = torch.addmm(self.bias, x, self.kernel)  # bias in the GEMM epilogue
            if self.activation is torch.relu:
                return torch.relu_(y)
        else:
            y = torch.matmul(x, self.kernel)
            if self.use_bias:
                y = y + self.bias
        if self.activation is not None:
            y = self.activation(y)
        return y


class Sequential(Layer):
    """keras.Sequential of Dense layers (GINConv's MLP, gin_conv.py:129-162)."""

    def __init__(self, layers: list[Layer], **kwargs):
        super().__init__(**kwargs)
        self.layers = torch.nn.ModuleList(layers)

    def build(self, input_shape) -> None:
        shape = tuple(input_shape)
        for layer in self.layers:
            if isinstance(layer, Dense) and not layer.built:
                layer._build_device = getattr(self, "_build_device", None)
                layer.build(shape)
                shape = shape[:-1] + (layer.units,)
        self.built = True

    def forward(self, x, training=None):
        if not self.built:
            self._build_device = x.device
            self.build(tuple(x.shape))
        for layer in self.layers:
            if isinstance(layer, Dropout):
                x = layer(x, training=training)
            else:
                x = layer(x)
        return x


class Dropout(Layer):
    def __init__(self, rate: float, **kwargs):
        super().__init__(**kwargs)
        self.rate = float(rate)

    def forward(self, x, training=None):
        if training and self.rate > 0:
            return torch.nn.functional.dropout(x, self.rate, training=True)
        return x
