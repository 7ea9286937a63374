"""Launch each SURVEY 8f kernel a few times for a rocprofv3 --kernel-trace
--stats pass (profiles/r01/next_rows_kernel_stats.csv): rcbf_gp_predict
(cars, N = 3000, B = 4096), rcbf_model_step (B = 65536), the replay ring
scatter / gather (65536 records), rcbf_obs_safe_action (+ backward, B = 256)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv  # noqa: E402


class A:
    cuda = True


env = BatchedSimulatedCarsEnv(4096, device=dev)
layer = CBFQPLayer(env, A(), gamma_b=20.0)
print(bench.sac_update_safe_action(env, layer, dev))
print(bench.next_rows(dev))
