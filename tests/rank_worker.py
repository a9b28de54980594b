"""One rank of tests/test_gpu_multirank.py: RANK/WORLD_SIZE/LOCAL_RANK and
MASTER_* come from the environment (set by the parent before this process
starts), as under torchrun.  The rank owns the contiguous slice
get_data_slice_multirank(N, rank, world) of a seeded N-image stream
(generator_files.rs:24-42), decodes + bucket-resizes it through its own
dg_ctx on device LOCAL_RANK mod the device count, and writes the outputs to
<out>/rank<r>.npz for the parent to check.

    rank_worker.py OUT_DIR N [SIZE RATIO]   (bucket config, default 512/16)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_dir: str, n: int, size: int = 512, ratio: int = 16) -> int:
    import torch
    import torch.distributed as dist

    from datago_amd import _lib as L
    from datago_amd import synth
    from datago_amd.sharding import get_data_slice_multirank
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = get_data_slice_multirank(n, rank, world)
    datas = synth.mixed_corpus(11, n, 96, 640, lo=lo, hi=hi)
    dev = local % torch.cuda.device_count()
    ctx = L.Context(dev, crop_and_resize=True, default_image_size=size, downsampling_ratio=ratio,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    res = ctx.decode_batch(datas)
    dist.barrier()
    arrays = {f"img{lo + k}": arr for k, (st, arr, meta) in enumerate(res) if st == 0}
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), device=np.array(dev),
             status=np.array([st for st, _, _ in res]), indices=np.arange(lo, hi), **arrays)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2]), *[int(x) for x in sys.argv[3:5]]))
