"""`_freqencoder` backend module: reference pybind11 surface
(freqencoder/src/freqencoder.h:6-9, f32 only as freqencoder.cu:109) over the
gfx950 C-ABI."""
import torch

from _dfhip import call, ptr, stream, checked


def _f32(t, what):
    checked(t, what)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{what} must be a float32 tensor")


def freq_encode_forward(inputs, B, D, deg, C, outputs):
    _f32(inputs, "inputs")
    _f32(outputs, "outputs")
    call("dfhip_freq_encode_forward", ptr(inputs), B, D, deg, C, ptr(outputs), stream())


def freq_encode_backward(grad, outputs, B, D, deg, C, grad_inputs):
    _f32(grad, "grad")
    _f32(outputs, "outputs")
    _f32(grad_inputs, "grad_inputs")
    call("dfhip_freq_encode_backward", ptr(grad), ptr(outputs), B, D, deg, C, ptr(grad_inputs),
         stream())
