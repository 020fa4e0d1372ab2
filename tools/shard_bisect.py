"""Run test_sharded_step_world1_bitwise_equals_fused under each combination of the row-sharded
step's launch-folding switches (distributed.GSUM_APPLY / GRAD_ROWS / BACK_ROWS / CLAIM_AHEAD) and report which
hold the bits (GPU only).
    python tools/shard_bisect.py"""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _ncf_pkg  # noqa: E402

_ncf_pkg.load()
import ncf_amd.distributed as Dist  # noqa: E402
from tests import test_gpu_parity as T  # noqa: E402

for gsum, grows, brows, cla in ((1, 1, 1, 0), (1, 1, 1, 1)):
    Dist.GSUM_APPLY, Dist.GRAD_ROWS, Dist.BACK_ROWS = bool(gsum), bool(grows), bool(brows)
    Dist.CLAIM_AHEAD = bool(cla)
    for exchange, ahead in (("rccl", False), ("rccl", True)):
        try:
            T.test_sharded_step_world1_bitwise_equals_fused(exchange, ahead)
            res = "ok"
        except Exception as e:   # noqa: BLE001
            res = "FAIL " + (str(e).splitlines() or [type(e).__name__])[0][:160]
            traceback.print_exc(limit=1)
        print(f"gsum={gsum} grad_rows={grows} back_rows={brows} claim_ahead={cla} {exchange} "
              f"ahead={ahead}: {res}",
              flush=True)
