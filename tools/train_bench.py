"""Time (and, under rocprofv3, trace) the training-step secondary workload of bench.py alone."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

import bench  # noqa: E402

if os.environ.get('NO_REPACK'):  # A/B: pack before every training forward instead of HipAdam's repack
    from chemprop_amd import train
    train.ADAM_REPACK = False
print(json.dumps(bench.training_workload(torch.device('cuda:0'), steps=int(os.environ.get('STEPS', '100')))))
