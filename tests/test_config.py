"""Config plumbing (transmil_deepgraft_amd/config.py): the reference's YAML keys
(Model.*, General.precision / grad_acc, Optimizer.*, Loss.*, Data.feature_extractor) mapped
onto the models, the compute dtype and the task, as code/train.py uses them."""
import pytest
import torch

YAML = """
General:
    seed: 2021
    precision: 16
    grad_acc: 2
Data:
    feature_extractor: retccl
Model:
    name: TransMIL
    n_classes: 3
    backbone: features
    in_features: 1024
    out_features: 512
Optimizer:
    opt: lookahead_radam
    lr: 0.0003
    weight_decay: 0.01
Loss:
    base_loss: CrossEntropyLoss
"""


def test_config_maps_reference_keys(tmp_path):
    from transmil_deepgraft_amd import config
    p = tmp_path / "TransMIL_test.yaml"
    p.write_text(YAML)
    cfg = config.read_yaml(p)
    assert cfg.Model.name == "TransMIL" and cfg.Data.mixup is None        # absent keys read as None
    assert config.compute_dtype_for(cfg.General.precision) == torch.bfloat16
    assert config.compute_dtype_for("32") == torch.float32
    with pytest.raises(ValueError):
        config.compute_dtype_for("64")
    assert config.in_features_of(cfg) == 2048                              # train.py:392-397
    model = config.build_model(cfg, device="cpu")
    assert model.n_classes == 3 and model.in_features == 2048 and model.compute_dtype == torch.bfloat16
    task = config.build_task(cfg, model)
    assert task.accumulate_grad_batches == 2 and task.lr == 3e-4
    assert config.build_task(cfg, model, n_gpus=8).accumulate_grad_batches == 10   # train.py:199
    cfg.Model.name = "Chowder"
    with pytest.raises(ValueError, match="not on the MI355X path"):
        config.build_model(cfg, device="cpu")
