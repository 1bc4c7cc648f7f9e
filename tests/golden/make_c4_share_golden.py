"""Freezes C4's real rank shares for tests/test_gpu_parity.py
test_c4_rank_share_block_path: the oracle's (oracle/oracle.cpp, pinned to the
unmodified reference by tests/test_oracle_golden.py) per-sample values of the
C3 scene at 1920x1080 on 1536 hashed pixels for samples 0..1023, summed in the
fast order's 32-sample blocks per rank share (ranks 0 and 1 of 8: samples
0..511 and 512..1023).  ~2 min on 8 cores.

    python tests/golden/make_c4_share_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle_py as O  # noqa: E402
from pathtrace import scenes  # noqa: E402
from pathtrace.scene import to_text  # noqa: E402
from test_gpu_parity import block_sum  # noqa: E402


def main():
    cfg = scenes.CONFIGS["C4"]
    share = cfg.spp // 8
    pix = np.sort(np.random.default_rng(44).choice(cfg.width * cfg.height, 1536, replace=False)).astype(np.int32)
    per = O.render(to_text(cfg.scene(), "/tmp/pt_c4_golden_img"), cfg.width, cfg.height, 2 * share, cfg.depth,
                   screen=cfg.screen, pixels=pix, order=O.ORDER_FAST, per_sample=True)
    sums = np.stack([block_sum(per[:, r * share:(r + 1) * share]) for r in (0, 1)])
    np.savez_compressed(os.path.join(HERE, "c4_shares.npz"), pixels=pix, sums=sums, both=block_sum(per),
                        meta=np.array([cfg.width, cfg.height, share, cfg.depth, 0x5EED], dtype=np.int64))
    print("c4_shares.npz", sums.shape)


if __name__ == "__main__":
    main()
