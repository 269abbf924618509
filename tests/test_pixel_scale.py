"""The pixel kernels' bf16 staging scales u8 pixels by a multiply with fl(1/255) instead of the
divide the reference's `obs / 255` performs (csrc/conv_pixel.h kInv255): after the bf16 rounding
every one of the 256 values must be bitwise the same."""
import numpy as np


def _bf16_rne(v: np.ndarray) -> np.ndarray:
    u = v.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF


def test_u8_scale_multiply_equals_divide_after_bf16():
    x = np.arange(256, dtype=np.float32)
    quotient = (x / np.float32(255)).astype(np.float32)
    product = (x * (np.float32(1) / np.float32(255))).astype(np.float32)
    assert np.array_equal(_bf16_rne(quotient), _bf16_rne(product))
    # the f32 values themselves differ for some x: the equality is a property of the rounding
    assert np.any(quotient != product)
