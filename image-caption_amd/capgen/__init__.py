"""capgen — MI355X-native caption-generator training engine (drop-in for the
Transformer path of shao-chi/Image-Caption).  Host code here; kernels in libcapgen.so."""
from .config import CapgenConfig, preset  # noqa: F401

__all__ = ["CapgenConfig", "preset", "Engine", "Transformer", "PolicyNetwork", "TRANSFORMER", "SelfCriticNetwork"]


def __getattr__(name):
    # lazy: importing the package must not require the shared library (CPU tests, build)
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name == "Transformer":
        from .model import Transformer
        return Transformer
    if name == "PolicyNetwork":
        from .model import PolicyNetwork
        return PolicyNetwork
    if name == "TRANSFORMER":
        from .models import TRANSFORMER
        return TRANSFORMER
    if name == "SelfCriticNetwork":
        from .models import SelfCriticNetwork
        return SelfCriticNetwork
    raise AttributeError(name)
