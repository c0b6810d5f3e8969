"""Native step program (csrc/hip/step_prog.hip): host-side validation of an
op list before any event or launch exists (no GPU needed)."""

import ctypes as C

import pytest


def _lib():
    try:
        from gentun_amd.ops import cnn_kernels as K
        return K, K.lib()
    except Exception as e:            # library not built in this checkout
        pytest.skip("libgentun_hip.so not loadable: {}".format(e))


def _ops(K, spec):
    ops = (K.ProgOp * len(spec))()
    for o, (kind, stream, event, v0) in zip(ops, spec):
        o.kind, o.stream, o.event = K.PROG_OPS[kind], stream, event
        o.v[0] = v0
    return ops


@pytest.mark.parametrize("spec,nev,nst", [
    ([("wait", 1, 0, 0), ("record", 0, 0, 0)], 1, 2),          # waited on before it is recorded
    ([("record", 2, 0, 0)], 1, 2),                              # stream index out of range
    ([("record", 0, 3, 0)], 1, 2),                              # event index out of range
    ([("gt_conv_fwd", 0, 0, 0)], 0, 1),                         # launch without an argument block
])
def test_invalid_programs_rejected(spec, nev, nst):
    K, L = _lib()
    ops = _ops(K, spec)
    assert not L.gt_prog_create(ops, len(spec), nev, nst)


def test_op_table_matches_library_abi():
    K, L = _lib()
    assert L.gt_sizeof_prog_op() == C.sizeof(K.ProgOp)
    assert sorted(K.PROG_OPS.values()) == list(range(len(K.PROG_OPS)))
    ops = _ops(K, [("record", 0, 0, 0)])
    ops[0].kind = len(K.PROG_OPS)                               # unknown kind
    assert not L.gt_prog_create(ops, 1, 1, 1)
