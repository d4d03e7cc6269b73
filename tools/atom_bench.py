"""Time (and, under rocprofv3, trace) the atom_messages secondary workload of bench.py alone."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.atom_messages_workload(torch.device('cuda:0'), steps=int(os.environ.get('STEPS', '100')))))
