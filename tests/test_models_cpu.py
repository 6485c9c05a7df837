"""Drop-in surface checks that need no GPU: constructors, attributes, state_dict keys
and shapes identical to the reference's (keys recorded in the golden fixtures), the
reference's parameter counts, and loud failure of the compute path on CPU tensors."""
import pytest
import torch

from cases import CASES, load_fixture


def _cls(kind):
    from models_fer_vit.image_vit import ImageViT
    from models_fer_vit.latent_vit import LatentViT
    from models_fer_vit.latent_vit_v2 import LatentViTv2

    return {"image_vit": ImageViT, "latent_vit": LatentViT, "latent_vit_v2": LatentViTv2}[kind]


@pytest.mark.parametrize("name", list(CASES))
def test_state_dict_keys_and_shapes_match_reference(name):
    c = CASES[name]
    m = _cls(c["kind"])(**c["ctor"])
    fx = load_fixture(name)
    sd = m.state_dict()
    assert list(sd.keys()) == [str(k) for k in fx["sd_keys"]]
    for (k, v), s in zip(sd.items(), fx["sd_shapes"]):
        assert ",".join(str(d) for d in v.shape) == str(s), k


def test_param_counts_match_survey():
    from models_fer_vit.image_vit import create_vit_base
    from models_fer_vit.latent_vit import LatentViT

    assert sum(p.numel() for p in create_vit_base().parameters()) == 85_804_039
    assert sum(p.numel() for p in LatentViT().parameters()) == 19_191_815


def test_encoder_layers_start_identical_like_torch_deepcopy():
    from models_fer_vit.latent_vit import LatentViT

    m = LatentViT(depth=3)
    a, b = m.transformer.layers[0], m.transformer.layers[2]
    assert torch.equal(a.self_attn.in_proj_weight, b.self_attn.in_proj_weight)
    assert torch.equal(a.linear1.weight, b.linear1.weight)


def test_hybrid_surface_and_freezing(capsys):
    from models_fer_vit.hybrid_latent_vit import RECOMMENDED_STRATEGIES, create_hybrid_latent_vit

    m = create_hybrid_latent_vit(model_size="tiny", use_pretrained=False, freeze_transformer=True, use_adapter=True,
                                 adapter_dim=64)
    keys = list(m.state_dict().keys())
    assert "transformer.0.attn.qkv.weight" in keys and "adapters.11.alpha" in keys and "head.2.weight" in keys
    assert m.pos_embed.shape == (1, 19, 192)
    assert all(not p.requires_grad for p in m.transformer.parameters())
    assert m.use_adapter and len(m.adapters) == 12
    assert set(RECOMMENDED_STRATEGIES) == {"full_finetune", "partial_freeze", "adapter", "linear_probe"}
    with pytest.raises(RuntimeError):
        create_hybrid_latent_vit(model_size="tiny", use_pretrained=True)


def test_cpu_forward_fails_loudly():
    from models_fer_vit.latent_vit import LatentViT

    with pytest.raises(RuntimeError, match="ROCm"):
        LatentViT(depth=1)(torch.randn(2, 18, 512))


def test_leam_config_helpers():
    from models_fer_vit.latent_vit_v2 import LatentViTv2

    m = LatentViTv2(depth=1, use_leam=True, use_spe=True)
    assert m.get_config() == {"model": "LatentViTv2", "use_lwn": False, "use_lwn_residual": False,
                              "use_spe": True, "use_leam": True}
    w = m.get_leam_weights()
    assert w.shape == (18,) and abs(float(w[5]) - float(torch.sigmoid(torch.tensor(1.0)))) < 1e-6
