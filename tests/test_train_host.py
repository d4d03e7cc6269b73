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
