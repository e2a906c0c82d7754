"""kvc_eager (kvcompress.utils.key_length_attention), checked independently of the goldens that
use it (CPU): on a compressed (ragged) cache its attention weights are the transformers 4.x
eager kernel's -- softmax(Q K^T * scaling + mask[..., :key_len]) built here by hand -- and on
layers of equal length the model's output and attention weights are the stock eager kernel's, bit
for bit.  (tests/golden/gen_eval_attention.py runs the reference's loop through kvc_eager, so a
bug there would appear in both the golden and the port; this pins it on its own.)"""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from kvcompress import utils as U  # noqa: E402

transformers = pytest.importorskip("transformers")


def _model(dtype=torch.float32, layers=2, heads=4, head_dim=32):
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM
    torch.manual_seed(0)
    cfg = GPTNeoXConfig(vocab_size=256, hidden_size=heads * head_dim, num_hidden_layers=layers,
                        num_attention_heads=heads, intermediate_size=4 * heads * head_dim,
                        rotary_pct=0.25, max_position_embeddings=512)
    cfg._attn_implementation = "eager"
    return GPTNeoXForCausalLM(cfg).to(dtype).eval()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ragged_layer_weights_match_hand_built_softmax(dtype):
    """A layer whose cache was compressed to key_len < the mask's length: kvc_eager cuts the mask
    to the first key_len columns, as transformers 4.x eager kernels did."""
    model = _model(dtype)
    attn = model.gpt_neox.layers[0].attention
    g = torch.Generator().manual_seed(1)
    B, H, q, d, kl, mlen = 1, 4, 3, 32, 11, 19
    Q = torch.randn(B, H, q, d, generator=g).to(dtype)
    K = torch.randn(B, H, kl, d, generator=g).to(dtype)
    V = torch.randn(B, H, kl, d, generator=g).to(dtype)
    mask = torch.zeros(B, 1, q, mlen, dtype=dtype)
    for i in range(q):  # a causal pattern over the uncompressed length, plus a masked column
        mask[:, :, i, mlen - q + i + 1:] = torch.finfo(dtype).min
    mask[:, :, :, 2] = torch.finfo(dtype).min
    out, w = U._eager_forward(attn, Q, K, V, mask, scaling=attn.scaling, dropout=0.0)
    # by hand: scores, the cut mask, fp32 softmax rounded to the dtype, weights @ V
    s = torch.matmul(Q, K.transpose(2, 3)) * attn.scaling + mask[..., :kl]
    w_ref = torch.softmax(s, dim=-1, dtype=torch.float32).to(dtype)
    assert torch.equal(w, w_ref)
    assert torch.equal(out, torch.matmul(w_ref, V).transpose(1, 2).contiguous())
    assert torch.all(w[..., 2] == 0)  # the masked column stays masked after the cut
    with pytest.raises(RuntimeError):  # the uncut mask does not fit (transformers 5 eager)
        torch.matmul(Q, K.transpose(2, 3)) * attn.scaling + mask


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_equal_length_layers_match_stock_eager(dtype):
    """Uncompressed (equal-length) layers: a forward pass under key_length_attention gives the
    stock eager kernel's logits and attention weights bit for bit, prefill and a cached step."""
    model = _model(dtype)
    ids = torch.tensor([[5, 17, 200, 3, 99, 42, 7, 1]])
    with torch.no_grad():
        ref = model(ids[:, :6], use_cache=True, output_attentions=True)
        ref2 = model(ids[:, 6:], past_key_values=ref.past_key_values, use_cache=True,
                     output_attentions=True)
        with U.key_length_attention(model, need_weights=True):
            assert model.config._attn_implementation == U.KEY_LENGTH_EAGER
            got = model(ids[:, :6], use_cache=True, output_attentions=True)
            got2 = model(ids[:, 6:], past_key_values=got.past_key_values, use_cache=True,
                         output_attentions=True)
    assert model.config._attn_implementation == "eager"  # restored
    for a, b in ((ref, got), (ref2, got2)):
        assert torch.equal(a.logits, b.logits)
        assert all(torch.equal(x, y) for x, y in zip(a.attentions, b.attentions))
