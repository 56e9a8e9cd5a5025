"""DP-SGD optimisers: per-microbatch gradients, summed (clipped for the Gaussian query), noised and
averaged, then the wrapped optimiser's update.

Reference: efls-train/python/efl/privacy/dp_optimizer.py
  GaussianSumQuery (:54-57) = tensorflow_privacy 0.3.0's (setup.py:26) with zero initial state:
    per record clip_by_global_norm(record, l2_norm_clip), sum, + N(0, stddev^2), stddev = clip * mult;
  ElementWiseGaussianSumQuery (:60-73): sum, then v + normal(shape) * v * noise_multiplier;
  make_optimizer_class (:80-220): compute_gradients splits the per-example loss into
    num_microbatches rows (:148-157; all rows when the batch does not divide), takes each row's
    gradient (:170-183), accumulates it through the query, noises the sums (:206-208) and divides
    by num_microbatches (:210-216);
  make_gaussian_optimizer_class (:224-256): ElementWise query without l2_norm_clip, Gaussian with it;
  DPAdagrad / DPAdam / DPGradientDescent (+ Gaussian) optimisers (:258-284).

The noise and the division run as ONE HIP kernel per variable (csrc/mask.hip efl_dp_noise: read the
sum once, write the averaged noised gradient once) with TF's normal construction (Philox4x32-10,
Box-Muller) from a per-process `NoiseStream`. The per-microbatch gradients are autograd's; the
clip is a torch reduction. No CPU fallback: the kernel needs the GPU.

Torch mapping. TF optimisers get their variables at minimize time; torch ones at construction.
These classes take either: `params` (as `params=`, or first positional with the DP arguments as
keywords, torch style: `DPAdamGaussianOptimizer(model.parameters(), noise_multiplier=1.0, lr=..)`),
or none (the reference's call shape, e.g. `DPGradientDescentGaussianOptimizer(noise_multiplier=1.0,
learning_rate=0.25)`), in which case the wrapped optimiser is built on the first
`compute_gradients` / `minimize` var_list. `learning_rate` is accepted for `lr`. Float64 (and
half-precision) variables train: their noise is TF's float32 normal cast to the variable's dtype,
and the clip norm is taken in float64 for float64 records.

One reference quirk is kept: each microbatch's loss is `reduce_func(tf.gather(loss, [i]), axis=0)`
(:172), a reduction over a length-1 axis, so 'mean' and 'sum' both leave the row as it is and its
gradient is that of the row's SUM (TF differentiates a non-scalar loss as its sum).
"""
from __future__ import annotations

import torch

from efl import errors, exporter, lib
from efl.privacy.secret_sharing import NoiseStream

_stream = NoiseStream()


@exporter.export("privacy.set_noise_seed")
def set_noise_seed(seed: int | None, counter: int = 0) -> None:
    """Fix (or, with None, re-randomise) this process's DP noise stream."""
    _stream.reset(seed, counter)


def noise_stream() -> NoiseStream:
    return _stream


def dp_noise(x: torch.Tensor, mode: int, sigma: float, divisor: float = 1.0, stream: NoiseStream | None = None):
    """efl_dp_noise over one float32 tensor: mode 0 (x + z x sigma) / divisor, mode 1
    (x + z sigma) / divisor, z ~ N(0, 1) drawn from `stream` (default: the process's)."""
    x = lib.as_tensor(x)
    if not x.dtype.is_floating_point:
        raise errors.InvalidArgumentError(f"DP noise needs a floating-point gradient, got {x.dtype}")
    if x.dtype != torch.float32:
        # the reference draws tf.random.normal(..., dtype=v.dtype); the kernel draws TF's float32
        # normal, so other float dtypes are noised in float32 and cast back (float64 variables keep
        # float32-accurate noise; parity with TF's noise stream is distributional either way)
        return dp_noise(x.float(), mode, sigma, divisor, stream).to(x.dtype)
    v, home = lib.on_device(x.detach())
    v = v.contiguous()
    if v.data_ptr() % 16:
        v = v.clone()
    seed, ctr0 = (stream or _stream).take(v.numel())
    out = torch.empty_like(v)
    lib.check(lib.raw().efl_dp_noise(v.data_ptr(), out.data_ptr(), v.numel(), int(mode), float(sigma),
                                     float(divisor), seed, ctr0, lib.stream_handle(v.device)))
    return lib.back(out, home)


def _zeros_like(t):
    return torch.zeros_like(t)


class _SumQuery:
    """DPQuery protocol (tensorflow_privacy dp_query.SumAggregationDPQuery) on lists of tensors."""

    def initial_global_state(self):
        return None

    def derive_sample_params(self, global_state):
        return None

    def initial_sample_state(self, template):
        return [_zeros_like(t) for t in template]

    def preprocess_record(self, params, record):
        return record

    def accumulate_record(self, params, sample_state, record):
        rec = self.preprocess_record(params, record)
        return [s + r for s, r in zip(sample_state, rec)]

    def get_noised_result(self, sample_state, global_state, divisor: float = 1.0):
        raise NotImplementedError


@exporter.export("privacy.GaussianSumQuery")
class GaussianSumQuery(_SumQuery):
    """Clip each record to l2_norm_clip (global norm over its tensors), sum, add N(0, stddev^2)
    (dp_optimizer.py:54-57; tensorflow_privacy 0.3.0 gaussian_query.GaussianSumQuery)."""

    def __init__(self, l2_norm_clip: float, stddev: float):
        self._l2_norm_clip = float(l2_norm_clip)
        self._stddev = float(stddev)

    def derive_sample_params(self, global_state):
        return self._l2_norm_clip

    def preprocess_record(self, params, record):
        # tf.clip_by_global_norm: t * clip * min(1 / ||record||, 1 / clip), in the record's dtype
        # (the widest of its tensors)
        dt = torch.float64 if any(t.dtype == torch.float64 for t in record) else torch.float32
        norm = torch.sqrt(sum((t.to(dt) * t.to(dt)).sum() for t in record))
        scale = params * torch.minimum(1.0 / norm, torch.tensor(1.0 / params, dtype=dt, device=norm.device))
        return [t * scale.to(t.dtype) for t in record]

    def get_noised_result(self, sample_state, global_state, divisor: float = 1.0):
        return [dp_noise(v, 1, self._stddev, divisor) for v in sample_state], global_state


@exporter.export("privacy.ElementWiseGaussianSumQuery")
class ElementWiseGaussianSumQuery(_SumQuery):
    """Sum, then v + normal(shape(v)) * v * noise_multiplier (dp_optimizer.py:60-73)."""

    def __init__(self, noise_multiplier: float = 1):
        self._noise_multiplier = float(noise_multiplier)

    def get_noised_result(self, sample_state, global_state, divisor: float = 1.0):
        return [dp_noise(v, 0, self._noise_multiplier, divisor) for v in sample_state], global_state


_DEFAULT_OPT_CONFIG = {"REDUCE": "mean"}


def _split_params(args, kwargs):
    """The torch optimiser's params if the caller gave them (first positional or `params=`)."""
    if "params" in kwargs:
        return kwargs.pop("params"), args
    if args and not isinstance(args[0], (int, float)):
        return args[0], args[1:]
    return None, args


def _bind(args, kwargs, *spec):
    """Bind the leading (name, default) parameters from positional args, then keywords; returns
    their values followed by the remaining positional args."""
    args = list(args)
    vals = []
    for name, default in spec:
        if args:
            if name in kwargs:
                raise TypeError(f"got multiple values for argument {name!r}")
            vals.append(args.pop(0))
        else:
            vals.append(kwargs.pop(name, default))
    return (*vals, tuple(args))


def _as_params(obj):
    """obj as a torch optimiser's params (a list of tensors or param-group dicts), or None when it
    is something else (a number, a query): lets `DPAdamGaussianOptimizer(model.parameters(), lr=..)`
    work although the reference's first positional argument is noise_multiplier."""
    if obj is None or isinstance(obj, (int, float, bool, str)) or hasattr(obj, "get_noised_result"):
        return None
    if isinstance(obj, torch.Tensor):
        return [obj]
    try:
        items = list(obj)
    except TypeError:
        return None
    if items and all(isinstance(t, (torch.Tensor, dict)) for t in items):
        return items
    return None


@exporter.export("privacy.make_optimizer_class")
def make_optimizer_class(cls):
    """A DP subclass of the torch optimiser class `cls` (dp_optimizer.py:80-220)."""

    class DPOptimizerClass(cls):
        def __init__(self, *args, **kwargs):
            """(dp_sum_query, num_microbatches=None, unroll_microbatches=False, [params], **opt
            kwargs), or torch style (params, dp_sum_query=..., ...)."""
            if "learning_rate" in kwargs:
                kwargs["lr"] = kwargs.pop("learning_rate")
            lead = _as_params(args[0]) if args else None
            if lead is not None:    # params first, torch style: the DP arguments are keywords then
                if "dp_sum_query" not in kwargs:
                    raise TypeError("params given first: pass dp_sum_query= as a keyword")
                kwargs["params"] = lead
                args = args[1:]
            dp_sum_query, num_microbatches, unroll_microbatches, args = _bind(
                args, kwargs, ("dp_sum_query", None), ("num_microbatches", None), ("unroll_microbatches", False))
            if dp_sum_query is None:
                raise TypeError("dp_sum_query is required")
            params, args = _split_params(args, kwargs)
            self._dp_sum_query = dp_sum_query
            self._num_microbatches = num_microbatches
            self._global_state = dp_sum_query.initial_global_state()
            self._unroll_microbatches = unroll_microbatches   # microbatches always run as a Python loop
            self._was_compute_gradients_called = False
            self._opt_args, self._opt_kwargs = args, kwargs
            self._built = False
            if params is not None:
                self._build(params)

        def _build(self, params):
            cls.__init__(self, params, *self._opt_args, **self._opt_kwargs)
            self._built = True

        def compute_gradients(self, loss, var_list=None, grad_loss=None, opt_config=None):
            """[(gradient, variable)] for a per-example loss tensor (first dim = batch)."""
            self._was_compute_gradients_called = True
            if callable(loss):
                raise NotImplementedError("Eager mode is not available yet")
            if var_list is None:
                if not self._built:
                    raise errors.InvalidArgumentError("var_list is required before the optimiser has params")
                var_list = [p for group in self.param_groups for p in group["params"]]
            var_list = list(var_list)
            if not self._built:
                self._build(var_list)
            opt_config = dict(_DEFAULT_OPT_CONFIG if opt_config is None else opt_config)
            reduce_func = opt_config.pop("REDUCE", "mean")
            if reduce_func not in ("mean", "sum") and not callable(reduce_func):
                raise ValueError("No such reduce function called '{}'.".format(str(reduce_func)))
            batch_size = int(loss.shape[0])
            nm = batch_size if self._num_microbatches is None else int(self._num_microbatches)
            if nm <= 0 or batch_size % nm != 0:
                nm = batch_size
            loss = loss.reshape(nm, -1)
            grad_loss = None if grad_loss is None else grad_loss.reshape(nm, -1)
            params = self._dp_sum_query.derive_sample_params(self._global_state)
            state = self._dp_sum_query.initial_sample_state([v.detach() for v in var_list])
            for i in range(nm):
                row = loss[i]
                if callable(reduce_func):
                    row = reduce_func(loss[i:i + 1], 0)
                # a non-scalar row differentiates as its sum (TF's gradients of a tensor loss)
                go = torch.ones_like(row) if grad_loss is None else grad_loss[i].reshape(row.shape)
                grads = torch.autograd.grad(row, var_list, grad_outputs=go, retain_graph=True, allow_unused=True)
                grads = [g if g is not None else torch.zeros_like(v) for g, v in zip(grads, var_list)]
                state = self._dp_sum_query.accumulate_record(params, state, grads)
            final, self._global_state = self._dp_sum_query.get_noised_result(state, self._global_state,
                                                                             divisor=float(nm))
            return list(zip(final, var_list))

        def apply_gradients(self, grads_and_vars):
            for g, v in grads_and_vars:
                v.grad = g.to(v.dtype)
            self.step()

        def minimize(self, loss, var_list=None, grad_loss=None, opt_config=None):
            self.apply_gradients(self.compute_gradients(loss, var_list, grad_loss, opt_config))

    DPOptimizerClass.__name__ = "DP" + cls.__name__
    return DPOptimizerClass


@exporter.export("privacy.make_gaussian_optimizer_class")
def make_gaussian_optimizer_class(cls):
    """A DP optimiser with Gaussian noise (dp_optimizer.py:224-256): element-wise noise scaled by
    each summed gradient without l2_norm_clip, clipped records + N(0, (clip * mult)^2) with it."""

    class DPGaussianOptimizerClass(make_optimizer_class(cls)):
        def __init__(self, *args, **kwargs):
            """(noise_multiplier=0, l2_norm_clip=None, num_microbatches=None,
            unroll_microbatches=False, [params], **opt kwargs), or torch style (params, ...)."""
            lead = _as_params(args[0]) if args else None
            if lead is not None:    # torch style: params first, the DP arguments as keywords
                kwargs["params"] = lead
                args = args[1:]
            noise_multiplier, l2_norm_clip, num_microbatches, unroll_microbatches, args = _bind(
                args, kwargs, ("noise_multiplier", 0), ("l2_norm_clip", None), ("num_microbatches", None),
                ("unroll_microbatches", False))
            if l2_norm_clip is None:
                q = ElementWiseGaussianSumQuery(noise_multiplier)
            else:
                q = GaussianSumQuery(l2_norm_clip, l2_norm_clip * noise_multiplier)
            super().__init__(q, num_microbatches, unroll_microbatches, *args, **kwargs)

        @property
        def ledger(self):
            return getattr(self._dp_sum_query, "ledger", None)

    DPGaussianOptimizerClass.__name__ = "DP" + cls.__name__ + "Gaussian"
    return DPGaussianOptimizerClass


# tf.train.{Adagrad, Adam, GradientDescent}Optimizer (dp_optimizer.py:258-260)
AdagradOptimizer = torch.optim.Adagrad
AdamOptimizer = torch.optim.Adam
GradientDescentOptimizer = torch.optim.SGD

DPAdagradOptimizer = exporter.export("privacy.DPAdagradOptimizer")(make_optimizer_class(AdagradOptimizer))
DPAdamOptimizer = exporter.export("privacy.DPAdamOptimizer")(make_optimizer_class(AdamOptimizer))
DPGradientDescentOptimizer = exporter.export("privacy.DPGradientDescentOptimizer")(
    make_optimizer_class(GradientDescentOptimizer))
DPAdagradGaussianOptimizer = exporter.export("privacy.DPAdagradGaussianOptimizer")(
    make_gaussian_optimizer_class(AdagradOptimizer))
DPAdamGaussianOptimizer = exporter.export("privacy.DPAdamGaussianOptimizer")(
    make_gaussian_optimizer_class(AdamOptimizer))
DPGradientDescentGaussianOptimizer = exporter.export("privacy.DPGradientDescentGaussianOptimizer")(
    make_gaussian_optimizer_class(GradientDescentOptimizer))
