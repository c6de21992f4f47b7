"""ctypes binding of libwam_hip.so (the C-ABI declared in include/wam_hip.h).

The library is loaded eagerly and the import FAILS LOUDLY when it is missing: there is no CPU or
PyTorch fallback for any WAM op. torch is imported first so that libwam_hip.so binds to the
libamdhip64.so.7 torch already loaded (one HIP runtime per process).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WAM_LIB_PATH") or os.path.join(_HERE, "libwam_hip.so")  # override: experiments
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "wam_hip.h")

if not os.path.exists(LIB_PATH):
    raise ImportError("wam_amd: %s is missing -- build it with `python -m wam_amd.build` "
                      "(hipcc --offload-arch=gfx950). There is no CPU fallback." % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p
c_dp = ctypes.POINTER(ctypes.c_double)
c_i64p = ctypes.POINTER(ctypes.c_int64)

_SIGS = {
    "wam_strerror": (ctypes.c_char_p, [c_int]),
    "wam_version": (c_int, []),
    "wam_plan_create": (c_int, [ctypes.POINTER(c_vp), c_int, c_i64p, c_int, c_dp, c_dp, c_dp, c_dp, c_int, c_int]),
    "wam_plan_create_ex": (c_int, [ctypes.POINTER(c_vp), c_int, c_i64p, c_int, c_dp, c_dp, c_dp, c_dp, c_int, c_int,
                                   c_int]),
    "wam_plan_destroy": (None, [c_vp]),
    "wam_plan_create_host": (c_int, [ctypes.POINTER(c_vp), c_int, c_i64p, c_int, c_dp, c_dp, c_dp, c_dp, c_int,
                                     c_int, c_int]),
    "wam_plan_num_bands": (c_int, [c_vp]),
    "wam_plan_band_shape": (c_int, [c_vp, c_int, c_i64p]),
    "wam_plan_band_offset": (c_i64, [c_vp, c_int]),
    "wam_plan_coeff_numel": (c_i64, [c_vp]),
    "wam_plan_rec_shape": (c_int, [c_vp, c_i64p]),
    "wam_plan_workspace_bytes": (c_i64, [c_vp, c_i64]),
    "wam_wavedec": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "wam_waverec": (c_int, [c_vp, c_i64, c_vp, ctypes.POINTER(c_f32), c_int, c_vp, c_vp, c_vp]),
    "wam_waverec_adjoint": (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "wam_item_sigma": (c_int, [c_i64, c_i64, c_i64, c_vp, c_f32, c_vp, c_vp]),
    "wam_item_sigma_ws_bytes": (c_i64, [c_i64, c_i64]),
    "wam_item_sigma_ws": (c_int, [c_i64, c_i64, c_i64, c_vp, c_f32, c_vp, c_vp, c_i64, c_vp]),
    "wam_noise_add": (c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, ctypes.c_uint64, c_i64, c_vp, c_vp]),
    "wam_noise_add_ex": (c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, ctypes.c_uint64, c_i64, c_i64, c_vp,
                                 c_vp]),
    "wam_subband_maps": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp]),
    "wam_frame_accumulate": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_vp, c_vp]),
    "wam_frame_accumulate_coef": (c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp,
                                          c_vp]),
    "wam_frame_trapz": (c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_int, c_vp, c_vp,
                                c_vp, c_vp]),
    "wam_frame_trapz_coef": (c_int, [c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp,
                                     c_vp, c_vp, c_vp]),
    "wam_cube_accumulate": (c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_int, c_f32, c_vp, c_vp, c_vp,
                                    c_vp]),
    "wam_accumulate_f32": (c_int, [c_i64, c_i64, c_vp, c_f32, c_vp, c_vp]),
    "wam_trapz_f32": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wam_reproject_scales": (c_int, [c_i64, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "wam_disentangle_scales": (c_int, [c_vp, c_i64, c_vp, c_vp, c_int, c_int, c_vp, c_vp]),
    "wam_plan_caps": (c_int, [c_vp]),
    "wam_wavedec_noisy": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, ctypes.c_uint64, c_i64, c_vp, c_vp, c_vp]),
    "wam_wavedec_noisy_ex": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, ctypes.c_uint64, c_i64, c_i64, c_vp, c_vp,
                                     c_vp]),
    "wam_waverec_adjoint_maps": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wam_waverec_bf16_nhwc": (c_int, [c_vp, c_i64, c_vp, ctypes.POINTER(c_f32), c_int, c_int, c_vp, c_vp]),
    "wam_waverec_adjoint_maps_bf16_nhwc": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp]),
    "wam_waverec_adjoint_maps_bf16": (c_int, [c_vp, c_i64, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "wam_timing_enable": (c_int, [c_int]),
    "wam_copy": (c_int, [c_i64, c_vp, c_vp, c_vp]),
    "wam_visualize3d": (c_int, [c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "wam_melspec": (c_int, [c_i64, c_i64, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wam_melspec_adjoint": (c_int, [c_i64, c_i64, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wam_rank_masks": (c_int, [c_i64, c_i64, c_i64, c_vp, c_int, c_vp, c_vp]),
    "wam_coeff_masks": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "wam_quantize_normalize": (c_int, [c_i64, c_int, c_i64, c_vp, ctypes.POINTER(c_f32), ctypes.POINTER(c_f32),
                                       c_vp, c_vp]),
    "wam_quantize_resize_normalize": (c_int, [c_i64, c_int, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp, c_vp,
                                              c_int, c_vp, c_vp, c_int, c_int, ctypes.POINTER(c_f32),
                                              ctypes.POINTER(c_f32), c_vp, c_vp, c_vp]),
    "wam_gaussian_filter2d": (c_int, [c_i64, c_int, c_int, c_dp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "wam_upsample_masks": (c_int, [c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "wam_masked_sums": (c_int, [c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "wam_ew_bias_act": (c_int, [c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_int, c_vp]),
    "wam_ew_add_bias_relu": (c_int, [c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wam_ew_relu_mask": (c_int, [c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wam_ew_maxpool_nhwc": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    "wam_ew_maxpool_nhwc_backward": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_vp, c_vp,
                                             c_int, c_vp, c_vp]),
    "wam_timing_drain": (c_int, [c_int, ctypes.c_char_p, ctypes.POINTER(c_f32), ctypes.POINTER(ctypes.c_double)]),
}

for _name, (_res, _args) in _SIGS.items():
    _fn = getattr(lib, _name)  # AttributeError here = the .so does not export a header symbol
    _fn.restype = _res
    _fn.argtypes = _args


class WamError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise WamError(lib.wam_strerror(rc).decode())
    return rc


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return c_vp(t.data_ptr())


def stream_of(device):
    return c_vp(torch.cuda.current_stream(device).cuda_stream)


def require_cuda(t, what="tensor"):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError("wam_amd: %s must be a CUDA (HIP) tensor; the WAM kernels run on the GPU only" % what)
    if t.dtype != torch.float32:
        raise TypeError("wam_amd: %s must be float32, got %s" % (what, t.dtype))
    return t
