"""k_apply launched alone, back to back (diagnostic tool): the r1w2 stream (read G, write the
residual in place and the output) through psgd_reconstruct, vs the same pass inside codec steps.
usage: python tools/apply_alone.py"""
import torch

from powersgd_amd import _lib
from powersgd_amd.reducers import _Codec

SETS = {
    "one (49152,512)": [(49152, 512)],
    "one (5120,4608)": [(5120, 4608)],
    "m512  (2048,512)x24": [(2048, 512)] * 24,
    "m4608 (512,4608)x10": [(512, 4608)] * 10,
    "m576  (4096,576)x10": [(4096, 576)] * 10,
}


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for name, shapes in SETS.items():
        for rank in (1, 4):
            g = [torch.randn(sh, device=dev) for sh in shapes]
            out = [torch.empty(sh, device=dev) for sh in shapes]
            c = _Codec(g, rank)
            c.P.normal_()
            c.Q.normal_()
            gp, op = c.ptrs(g), c.ptrs(out)
            term = (c.P.data_ptr(), c.Q.data_ptr())
            for _ in range(3):
                c.plan.reconstruct(gp, gp, op, [term], [term], 1.0, s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            n = 50
            for _ in range(n):
                c.plan.reconstruct(gp, gp, op, [term], [term], 1.0, s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / n * 1e3
            nb = sum(x.numel() for x in g) * 4
            print(f"{name} r{rank}: k_apply alone {us:7.2f} us  {3 * nb / us / 1e3:6.0f} GB/s", flush=True)
            del g, out, c
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
