"""a5 static-context input (train.py:92-113, 154-158): g2k_context_conv_f32
vs the float64 restatement (oracle.context_conv, static_mask, context_input).
Parity unpinned against the reference (unseeded random filter, ctxt.png
absent).  Tolerance (written here): normwise 1e-4 (sums of ~1e6 products)."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import context
from oracle import g2k_ref as ref


def test_filter_shape_matches_reference_formula():
    # train.py:100-106: width/height of the padded image, filter [w-dim+1, h-dim+1]
    assert context.context_filter_shape(576, 720, 3, 16) == (576 + 2 - 15, 720 + 1 - 15, 3)


def test_cpu_tensor_rejected():
    with pytest.raises(ValueError):
        context.static_context(torch.zeros(20, 20, 3))


@pytest.mark.gpu
@pytest.mark.parametrize("h,w,c,dim", [(30, 41, 3, 16), (17, 16, 1, 10), (120, 200, 3, 16)])
def test_context_conv_matches_oracle(gpu, h, w, c, dim):
    rng = np.random.default_rng(h + w)
    img = rng.uniform(0, 255, size=(h, w, c)).astype(np.float32)
    filt = rng.standard_normal(context.context_filter_shape(h, w, c, dim)).astype(np.float32)
    conv, G = context.static_context(torch.from_numpy(img).to(gpu),
                                     torch.from_numpy(filt).to(gpu), dim=dim, lam=5e-4)
    torch.cuda.synchronize()
    rc = ref.context_conv(img, filt, dim, 5e-4)
    rG = ref.context_input(rc, ref.static_mask(dim, 8))
    assert np.abs(conv.cpu().numpy() - rc).max() <= 1e-4 * np.abs(rc).max()
    assert np.abs(G.cpu().numpy() - rG).max() <= 1e-4 * np.abs(rG).max()


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [16, 10])
def test_context_conv_full_frame(gpu, dim):
    """The reference's frame size (576 x 720 x 3, padded to 578 x 721,
    train.py:95-110): a 563 x 706 x 3 filter at D = 16 (569 x 712 at D = 10)."""
    rng = np.random.default_rng(dim)
    img = rng.uniform(0, 255, size=(576, 720, 3)).astype(np.float32)
    filt = rng.standard_normal(context.context_filter_shape(576, 720, 3, dim)).astype(np.float32)
    conv, G = context.static_context(torch.from_numpy(img).to(gpu), torch.from_numpy(filt).to(gpu),
                                     dim=dim, lam=5e-4)
    torch.cuda.synchronize()
    rc = ref.context_conv(img, filt, dim, 5e-4)
    rG = ref.context_input(rc, ref.static_mask(dim, 8))
    assert np.abs(conv.cpu().numpy() - rc).max() <= 1e-4 * np.abs(rc).max()
    assert np.abs(G.cpu().numpy() - rG).max() <= 1e-4 * np.abs(rG).max()
