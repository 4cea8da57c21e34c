"""Host-side checks of the sibling heads (no GPU): every drop-in model exposes exactly the
reference's state_dict keys and shapes (via the pinned oracle restatements), and refuses CPU
tensors instead of falling back."""
import pytest
import torch

from golden_util import index
from test_oracle import SIBLINGS, sibling_oracle


@pytest.mark.parametrize("name", SIBLINGS)
def test_sibling_state_dict_layout(name):
    from transmil_deepgraft_amd import models
    meta = index()[name]
    ours = getattr(models, meta["model"])(**meta["ctor"])
    ref = sibling_oracle(name)
    a = {k: tuple(v.shape) for k, v in ours.state_dict().items()}
    b = {k: tuple(v.shape) for k, v in ref.state_dict().items()}
    assert a == b
    with pytest.raises(RuntimeError, match="GPU"):
        ours(torch.zeros(tuple(meta["input_shape"])))


def test_attention_map_refuses_huge_materialisation():
    """The lazy return_attn product raises instead of allocating B*h*n'^2 fp32 above the limit
    (35 GB per layer at N = 32768); row access stays available."""
    from transmil_deepgraft_amd.nystrom_attention import AttentionMap
    qkv = torch.empty(3, 8, 33280, 64, device="meta")
    attn = AttentionMap(qkv, {}, heads=8)
    assert tuple(attn.shape) == (1, 8, 33280, 33280)
    with pytest.raises(RuntimeError, match="GiB"):
        attn.full()
    with pytest.raises(RuntimeError, match="GiB"):
        attn[:, :, 5:7]
