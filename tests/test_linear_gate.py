"""the TN weight-gradient gate of ops/linear.py mirrors the
kernel's operand contract (csrc/gemm/gemm_xl.hip check_bf16_2d), so views the
kernel would reject take the library path instead of raising in backward."""
import torch

from distributed_model_parallel_amd.ops.linear import _gemm_operand_ok


def test_gemm_operand_contract():
    base = torch.zeros(64, 512, dtype=torch.bfloat16)
    assert _gemm_operand_ok(base)
    assert _gemm_operand_ok(base[:, 256:])              # 512-B offset: 16-B aligned
    assert not _gemm_operand_ok(base[:, 3:259])         # 6-B offset: misaligned base
    assert not _gemm_operand_ok(base.t())               # column stride != 1
    assert not _gemm_operand_ok(base.float())           # dtype
    odd = torch.zeros(64, 260, dtype=torch.bfloat16)[:, :256]
    assert not _gemm_operand_ok(odd)                    # row stride 260: rows not 16-B aligned
