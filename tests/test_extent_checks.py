"""Operand extents are checked before any launch (_hip.gemm_args / attn_set):
the kernels take plain pointers and strides, so an oversize M, K or row stride
from a caller would read or write past an allocation on the device.  These run
on CPU tensors: the checks only look at the storage, nothing is launched."""
import pytest
import torch

from neurosync_trainer_lite_amd import _hip as K

bf = torch.bfloat16


def _gemm(M, N, Kd, A=None, B=None, C=None, **kw):
    A = torch.zeros(M, Kd, dtype=bf) if A is None else A
    B = torch.zeros(N, Kd, dtype=bf) if B is None else B
    C = torch.zeros(M, N, dtype=bf) if C is None else C
    return K.gemm_args(A, B, C, M, N, Kd, **kw)


def test_gemm_args_in_bounds():
    a = _gemm(512, 256, 128)
    assert (a.M, a.N, a.K, a.lda, a.ldb, a.ldc) == (512, 256, 128, 128, 128, 256)
    # a column window of a wider matrix: its last row ends inside the storage
    X = torch.zeros(512, 3 * 128, dtype=bf)
    _gemm(512, 256, 128, A=X[:, 128:256])
    # MN-major operands ([K][M], [K][N])
    K.gemm_args(torch.zeros(128, 512, dtype=bf), torch.zeros(128, 256, dtype=bf), torch.zeros(512, 256),
                512, 256, 128, a_kmajor=False, b_kmajor=False)


@pytest.mark.parametrize("what", ["M", "K", "N", "lda", "ldc"])
def test_gemm_args_oversize_raises(what):
    M, N, Kd = 512, 256, 128
    kw = {}
    if what == "M":
        M = 513
        A, C = torch.zeros(512, Kd, dtype=bf), torch.zeros(513, N, dtype=bf)
        with pytest.raises(ValueError, match="A"):
            _gemm(M, N, Kd, A=A, C=C)
        return
    if what == "K":
        with pytest.raises(ValueError, match="A"):
            _gemm(M, N, Kd + 64, A=torch.zeros(M, Kd, dtype=bf), B=torch.zeros(N, Kd + 64, dtype=bf))
        return
    if what == "N":
        with pytest.raises(ValueError, match="C"):
            _gemm(M, N + 256, Kd, B=torch.zeros(N + 256, Kd, dtype=bf), C=torch.zeros(M, N, dtype=bf))
        return
    if what == "lda":
        kw["lda"] = 136
    else:
        kw["ldc"] = 264
    with pytest.raises(ValueError):
        _gemm(M, N, Kd, **kw)


def test_gemm_args_window_past_the_end_raises():
    # the last 128 columns of a [512][384] matrix read as K = 192 run past its end
    X = torch.zeros(512, 384, dtype=bf)
    with pytest.raises(ValueError, match="A"):
        _gemm(512, 256, 192, A=X[:, 256:], B=torch.zeros(256, 192, dtype=bf))


def test_gemm_args_side_outputs():
    M, N, Kd = 512, 256, 128
    with pytest.raises(ValueError, match="bias"):
        _gemm(M, N, Kd, bias=torch.zeros(N - 1))
    with pytest.raises(ValueError, match="relu_mask"):
        _gemm(M, N, Kd, relu_mask=torch.zeros(((M + 63) // 64) * 8 * (N // 8) - 1, dtype=torch.int64))
    with pytest.raises(ValueError, match="colsum"):
        _gemm(M, N, Kd, colsum_part=torch.zeros(M // 128 - 1, N))
    with pytest.raises(ValueError, match="aux"):
        _gemm(M, N, Kd, aux=torch.zeros(M - 1, N, dtype=bf), ld_aux=N)
    with pytest.raises(ValueError, match="rope"):
        _gemm(M, N, Kd, rope=(torch.zeros(128, 31), torch.zeros(128, 32), 128, 64))
    _gemm(M, N, Kd, bias=torch.zeros(N), colsum_part=torch.zeros(M // 128, N),
          relu_mask=torch.zeros(((M + 63) // 64) * 8 * (N // 8), dtype=torch.int64))


def _attn(B=2, T=128, H=4, dh=64):
    return K.attn_args(K.BF16, B, T, H, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.0, 0, dh=dh)


def test_attn_set_in_bounds_and_strides():
    B, T, H, dh = 2, 128, 4, 64
    D = H * dh
    qkv = torch.zeros(B * T, 3 * D, dtype=bf)
    a = K.attn_set(_attn(), q=qkv[:, :D], k=qkv[:, D:2 * D], v=qkv[:, 2 * D:], o=torch.zeros(B * T, D, dtype=bf),
                   lse=torch.zeros(B * H * T), mask_bits=torch.zeros(B * H * T * T // 64, dtype=torch.int64))
    assert (a.q_ld, a.k_ld, a.v_ld, a.o_ld) == (3 * D, 3 * D, 3 * D, D)
    assert a.v == qkv[:, 2 * D:].data_ptr()


def test_attn_set_oversize_raises():
    B, T, H, dh = 2, 128, 4, 64
    D = H * dh
    with pytest.raises(ValueError, match="q"):
        K.attn_set(_attn(), q=torch.zeros(B * T - 1, D, dtype=bf))
    with pytest.raises(ValueError, match="lse"):
        K.attn_set(_attn(), lse=torch.zeros(B * H * T - 1))
    with pytest.raises(ValueError, match="mask_bits"):
        K.attn_set(_attn(), mask_bits=torch.zeros(B * H * T * T // 64 - 1, dtype=torch.int64))
    qkv = torch.zeros(B * T, 3 * D, dtype=bf)
    with pytest.raises(ValueError, match="v"):
        K.attn_set(_attn(), v=qkv[:, 2 * D + 64:])  # the window's last row runs past the end
    with pytest.raises(TypeError):
        K.attn_set(_attn(), qq=qkv)
