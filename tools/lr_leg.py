"""Measurement helper: bench.py's config-2 leg (local_reduce) alone, printed as JSON."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "oxidized-neural-orchestra_amd"))
import torch  # noqa: E402
import ono_amd  # noqa: E402
import bench  # noqa: E402

print(json.dumps(bench.local_reduce(torch, ono_amd, 20, 5)))
