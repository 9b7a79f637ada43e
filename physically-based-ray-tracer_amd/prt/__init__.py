"""prt -- MI355X-native path-tracing hot path (host-side mirror of the reference's
Renderer / Scene / Camera API; compute in hand-written HIP kernels behind include/prt.h)."""
from . import scenes, tiles
from ._lib import (FLAGS_DEFAULT, FLAG_AA, FLAG_ACCUMULATE, FLAG_GAMMA, FLAG_LIGHTED, FLAG_NORMALMAP, FLAG_SKYBOX,
                   FLAG_STOCHASTIC, PrtError, load)
from .renderer import Camera, Context, LightTransform, Renderer, Scene, postfx_preset

__all__ = ["scenes", "tiles", "load", "PrtError", "Camera", "Context", "LightTransform", "Renderer", "Scene",
           "FLAGS_DEFAULT", "FLAG_AA", "FLAG_ACCUMULATE", "FLAG_GAMMA", "FLAG_LIGHTED", "FLAG_NORMALMAP",
           "FLAG_SKYBOX", "FLAG_STOCHASTIC"]
