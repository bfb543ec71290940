"""zenflow_amd — MI355X-native (gfx950) drop-in for zenflow's neural spline
flow hot path: Flow.log_prob / sample over rolling spline couplings.

Public surface mirrors the reference package (src/zenflow/__init__.py):
``Flow``, ``train`` and the submodules ``bijectors``, ``distributions``,
``utils``; ``Module`` is the FLAX-style module protocol (``init`` / ``apply``,
submodules named by attribute, ``setup``, ``param`` / ``variable``) that user
modules holding a Flow build on.  All arithmetic runs in hand-written HIP kernels behind the C ABI
in include/zenflow_amd.h."""

from .flow import BoundFlow, Flow
from . import activations, bijectors, distributions, io, utils
from .io import load_variables, save_variables
from .module import Module, Variable
from .random import PRNGKey
from .train import Optimizer, adamw, nadamw, train

__all__ = "Flow", "train", "BoundFlow", "PRNGKey", "save_variables", "load_variables", "nadamw", "adamw", "Optimizer", "Module", "Variable"
