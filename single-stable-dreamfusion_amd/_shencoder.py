"""`_shencoder` backend module: reference pybind11 surface
(shencoder/src/shencoder.h:8-9) over the gfx950 C-ABI."""
import _dfhip as _d
from _dfhip import call, ptr, stream, checked


def sh_encode_forward(inputs, outputs, B, D, C, dy_dx):
    checked(inputs, "inputs")
    checked(outputs, "outputs")
    call("dfhip_sh_encode_forward", _d.dtype_code(inputs, "inputs"), ptr(inputs), ptr(outputs),
         B, D, C, ptr(dy_dx), stream())


def sh_encode_backward(grad, inputs, B, D, C, dy_dx, grad_inputs):
    for t, w in ((grad, "grad"), (inputs, "inputs"), (dy_dx, "dy_dx"),
                 (grad_inputs, "grad_inputs")):
        checked(t, w)
    call("dfhip_sh_encode_backward", _d.dtype_code(grad, "grad"), ptr(grad), ptr(inputs), B, D, C,
         ptr(dy_dx), ptr(grad_inputs), stream())
