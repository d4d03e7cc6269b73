"""CPU: host-side training plumbing (chemprop_amd/train.py) against its reference definitions."""
import math

import torch

from chemprop_amd.train import NoamLR, batch_loss, get_loss_func


def test_noam_schedule_matches_reference_formula():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=1e-4)
    s = NoamLR(opt, warmup_epochs=[2.0], total_epochs=[10], steps_per_epoch=5, init_lr=[1e-4], max_lr=[1e-3],
               final_lr=[1e-4])
    lrs = []
    for _ in range(60):
        s.step()
        lrs.append(opt.param_groups[0]['lr'])
    # the _LRScheduler constructor already took step 1 (as for the reference), so lrs[k] is step k + 2;
    # nn_utils.py:174-194: linear to max_lr at step 10, exponential decay to final_lr at step 50
    assert math.isclose(lrs[8], 1e-3, rel_tol=1e-9)
    assert math.isclose(lrs[3], 1e-4 + 5 * (9e-4 / 10), rel_tol=1e-9)
    assert math.isclose(lrs[48], 1e-4, rel_tol=1e-6)
    assert lrs[59] == 1e-4


def test_masked_weighted_loss():
    preds = torch.tensor([[1.0, 2.0], [3.0, 4.0]])
    targets = [[1.5, None], [2.0, 5.0]]
    loss = batch_loss(preds, targets, get_loss_func('regression'), data_weights=[1.0, 2.0])
    expect = (0.25 * 1 + (1.0 * 2 + 1.0 * 2)) / 3  # train.py:73-74
    assert math.isclose(float(loss), expect, rel_tol=1e-6)


def test_loss_matches_reference_formula_with_all_weights():
    """train.py:46-74 restated literally (mask / targets / target_weights / data_weights tensors, the
    product, loss.sum() / mask.sum()) against batch_loss's host-combined weight table: values and
    gradients."""
    g = torch.Generator().manual_seed(1)
    preds = torch.randn(6, 3, generator=g, requires_grad=True)
    tb = [[0.3, None, 1.2], [None, None, -0.4], [2.0, 0.1, 0.0], [0.5, -1.0, None], [1.0, 1.0, 1.0],
          [None, 0.7, 0.2]]
    tw, dw = [0.5, 2.0, 1.5], [1.0, 0.3, 2.5, 1.0, 0.7, 1.2]
    mask = torch.Tensor([[x is not None for x in r] for r in tb])
    targets = torch.Tensor([[0 if x is None else x for x in r] for r in tb])
    ref = (torch.nn.MSELoss(reduction='none')(preds, targets) * torch.Tensor(tw).unsqueeze(0)
           * torch.Tensor(dw).unsqueeze(1) * mask)
    ref = ref.sum() / mask.sum()
    g_ref, = torch.autograd.grad(ref, preds)
    out = batch_loss(preds, tb, get_loss_func('regression'), target_weights=tw, data_weights=dw)
    g_out, = torch.autograd.grad(out, preds)
    assert math.isclose(out.item(), ref.item(), rel_tol=1e-6)
    assert torch.allclose(g_out, g_ref, rtol=1e-6, atol=1e-8)


def test_loss_classification_and_multiclass():
    preds = torch.tensor([[0.5, -1.0], [2.0, 0.0]])
    targets = [[1, None], [0, 1]]
    loss = batch_loss(preds, targets, get_loss_func('classification'), dataset_type='classification')
    bce = torch.nn.functional.binary_cross_entropy_with_logits
    expect = (bce(preds[0, 0], torch.tensor(1.)) + bce(preds[1, 0], torch.tensor(0.))
              + bce(preds[1, 1], torch.tensor(1.))) / 3
    assert math.isclose(float(loss), float(expect), rel_tol=1e-6)
    logits = torch.randn(3, 1, 4, generator=torch.Generator().manual_seed(0))
    loss = batch_loss(logits, [[2], [0], [3]], get_loss_func('multiclass'), dataset_type='multiclass')
    expect = torch.nn.functional.cross_entropy(logits[:, 0, :], torch.tensor([2, 0, 3]))
    assert math.isclose(float(loss), float(expect), rel_tol=1e-6)


def test_build_optimizer_follows_reference_args():
    from chemprop_amd import TrainArgs
    from chemprop_amd.train import build_optimizer
    m = torch.nn.Linear(4, 2)
    opt = build_optimizer(m, TrainArgs(init_lr=3e-4, weight_decay=0.01, device=torch.device('cpu')))
    assert type(opt) is torch.optim.Adam
    assert opt.param_groups[0]['lr'] == 3e-4 and opt.param_groups[0]['weight_decay'] == 0.01
    opt = build_optimizer(m, TrainArgs(optimizer='adamw', device=torch.device('cpu')))
    assert type(opt) is torch.optim.AdamW and opt.param_groups[0]['lr'] == 1e-4
    assert build_optimizer(m, 2e-3).param_groups[0]['lr'] == 2e-3


def test_direct_step_requires_every_trainable_parameter_written():
    """the direct step skips zero_grad and writes only the encoder's native gradients and the
    fused head's; a model with any other trainable parameter must take the autograd path."""
    from chemprop_amd import MoleculeModel, TrainArgs, synthetic
    from chemprop_amd.featurization import BatchMolGraph
    from chemprop_amd.train import _direct_encoder
    model = MoleculeModel(TrainArgs(hidden_size=32, depth=3, device=torch.device('cpu')))
    head = (model.ffn[1], model.ffn[4], 0)
    batch = [BatchMolGraph(synthetic.make_batch('polymer', 2, 0))]
    assert _direct_encoder(model, batch, None, head) is model.encoder.encoder[0]
    model.extra = torch.nn.Parameter(torch.zeros(3))  # trainable, but no direct-step gradient
    assert _direct_encoder(model, batch, None, head) is None
    model.extra.requires_grad_(False)  # frozen parameters stop the direct path as before
    assert _direct_encoder(model, batch, None, head) is None
