"""vitmi — MI355X-native (gfx950) ViT forward/backward training path.

See DESIGN.md.  ``vitmi.modules`` holds the nn.Module API, ``vitmi.ops`` the
tensor wrappers over the C ABI in ``include/vitmi.h`` (``libvitmi.so``).
"""
from .config import ViTConfig, preset, config_c1, config_c2, config_c3, config_c5  # noqa: F401

__version__ = "0.1.0"


def _lazy():
    from . import modules, ops  # noqa: F401
    return modules, ops
