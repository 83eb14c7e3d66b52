"""CPU checks of the fp8 restatement (oracle/fp8_ref.py) the GPU fp8 path is
pinned to: OCP e4m3fn codes, round to nearest even, subnormals, the row-wise
scale rule, and the dequantized GEMM."""
import torch

from oracle import fp8_ref


def codes(vals):
    return torch.tensor(vals, dtype=torch.float32).to(torch.float8_e4m3fn).view(torch.uint8).tolist()


def test_e4m3fn_codes_round_to_nearest_even():
    # 1.0 = 0x38; 448 = 0x7E (largest finite); 2^-6 = smallest normal 0x08; 2^-9 = smallest subnormal 0x01
    assert codes([1.0, 448.0, 2.0 ** -6, 2.0 ** -9, -1.0]) == [0x38, 0x7E, 0x08, 0x01, 0xB8]
    # ties: 1.0625 lies halfway between 1.0 (mantissa 0) and 1.125 (1) -> 1.0;
    # 1.1875 halfway between 1.125 (1) and 1.25 (2) -> 1.25
    assert codes([1.0625, 1.1875]) == [0x38, 0x3A]


def test_quant_rows_scale_rule():
    x = torch.tensor([[0.0, 0.0, 0.0, 0.0], [1.0, -2.0, 0.5, 0.25], [3e-3, -1e-4, 0.0, 7.0]])
    q, s = fp8_ref.quant_rows(x)
    assert s[0].item() == 1.0 and (q[0].float() == 0).all()
    assert s[1].item() == torch.tensor(2.0 / 448.0).item()
    # the row maximum maps to +-448 exactly
    assert q[1].float()[1].item() == -448.0 and q[2].float()[3].item() == 448.0
    back = fp8_ref.dequant(q, s)
    assert torch.allclose(back[1:], x[1:], rtol=2 ** -4, atol=float(s[2]) * 2 ** -9)


def test_gemm_of_dequantized_operands():
    g = torch.Generator().manual_seed(0)
    a, b = torch.randn(8, 64, generator=g), torch.randn(5, 64, generator=g)
    qa, sa = fp8_ref.quant_rows(a)
    qb, sb = fp8_ref.quant_rows(b)
    ref = fp8_ref.dequant(qa, sa).double() @ fp8_ref.dequant(qb, sb).double().T
    assert torch.allclose(fp8_ref.gemm(qa, sa, qb, sb), ref, rtol=1e-6, atol=1e-5)  # dequant rounds in f32
    # e4m3 keeps ~3 mantissa bits: the product is within a few percent of the exact one
    rel = ((ref - a.double() @ b.double().T).norm() / (a.double() @ b.double().T).norm()).item()
    assert rel < 0.08
