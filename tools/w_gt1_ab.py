"""Times the world-size > 1 code path (1-rank RCCL group, bench.one_rank_group) for cfg3 and
cfg2 under the current environment; prints one JSON line. For A/B runs of plan knobs:
PSGD_FIN_ELEMS_KT=12000 python tools/w_gt1_ab.py"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

a = argparse.Namespace(steps=int(os.environ.get("AB_STEPS", "100")), warmup=10, sets=4, iters=None,
                       config="cfg3_resnet50_r4")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
r = bench.one_rank_group(a, dev)
def ms(v):
    if not isinstance(v, dict):
        return v
    return v["ms_per_step"] if "ms_per_step" in v else {k: ms(x) for k, x in v.items()}


print(json.dumps({k: ms(v) for k, v in r.items() if k != "note"}))
