"""zenflow_amd — MI355X-native (gfx950) drop-in for zenflow's neural spline
flow hot path: Flow.log_prob / sample over rolling spline couplings.

Public surface mirrors the reference package (src/zenflow/__init__.py):
``Flow``, ``train`` and the submodules ``bijectors``, ``distributions``,
``utils``.  All arithmetic runs in hand-written HIP kernels behind the C ABI
in include/zenflow_amd.h."""

from .flow import BoundFlow, Flow
from . import bijectors, distributions, io, utils
from .io import load_variables, save_variables
from .random import PRNGKey

__all__ = "Flow", "train", "BoundFlow", "PRNGKey", "save_variables", "load_variables"


def train(*args, **kwargs):
    """zenflow.train (train.py:18-138) — out of scope for this hot-path build.

    Training needs the spline/MLP backward pass and an optimiser; the GPU
    forward in train mode (batch statistics) exists (``apply(...,
    train=True, mutable=["batch_stats"])``), the gradient path does not yet."""
    raise NotImplementedError(
        "zenflow_amd.train: gradient-based training is not implemented "
        "(this build accelerates log_prob / sample; see DESIGN.md §Out of scope)"
    )
