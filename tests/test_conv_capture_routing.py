"""Round 4, profiles/README.md finding 48: inside a hipGraph capture the conv
routing leaves MIOpen out (its small-map weight gradient does not replay), and
eagerly conv_wgrad_xl takes layer-4-sized 3x3 weight gradients only up to
_XL_WGRAD_MAX_ROWS output pixels (MIOpen measured faster above)."""
from distributed_model_parallel_amd.ops import conv_igemm


def test_xl_wgrad_gate_by_rows_and_capture(monkeypatch):
    monkeypatch.setattr(conv_igemm, "_XL_WGRAD", True)
    monkeypatch.setattr(conv_igemm, "_capturing", lambda: False)
    small, big = conv_igemm._XL_WGRAD_MAX_ROWS, conv_igemm._XL_WGRAD_MAX_ROWS + 1
    assert conv_igemm._xl_wgrad_ok(512, 3, 3, small)        # layer 4 at batch 256: 12544 rows
    assert not conv_igemm._xl_wgrad_ok(512, 3, 3, big)      # batch 2048: MIOpen eagerly
    assert not conv_igemm._xl_wgrad_ok(128, 3, 3, small)    # Cin % 256 != 0: not this kernel
    assert not conv_igemm._xl_wgrad_ok(512, 1, 1, small)    # 1x1: the GEMM paths
    monkeypatch.setattr(conv_igemm, "_capturing", lambda: True)
    assert conv_igemm._xl_wgrad_ok(512, 3, 3, big)          # captured: never MIOpen


def test_generic_backward_env_default():
    # the generic native backward is opt-in eagerly (set_generic_backward); a
    # capture turns it on by itself
    assert conv_igemm.NATIVE_BWD in (False, True)
    assert callable(conv_igemm._capturing)
