"""trt-mi355x: an MI355X-native (gfx950) Whitted ray tracer with the hot path of
nobodyscool/vkComputeShader_tinyraytracer (shader.comp cast_ray) as a hand-written HIP
kernel behind a C-ABI (include/trt/abi.h)."""
from . import types
from ._lib import ABI_SYMBOLS, LIB_PATH, TrtError, lib
from .renderer import Renderer, render, write_image
from .scene import (
    CONFIGS,
    MODEL_INFOS,
    Scene,
    SceneBuilder,
    camera_path,
    config_c1,
    config_c2,
    config_c3,
    config_c4,
    config_c5,
    config_readme,
    config_reference_default,
    icosphere,
    make_ubo,
    synthetic_envmap,
)

__all__ = [
    "types", "ABI_SYMBOLS", "LIB_PATH", "TrtError", "lib", "Renderer", "render", "CONFIGS",
    "MODEL_INFOS", "Scene", "SceneBuilder", "camera_path", "config_c1", "config_c2", "config_c3", "config_c4",
    "config_c5", "config_readme", "config_reference_default", "icosphere", "make_ubo", "synthetic_envmap", "write_image",
]
