"""Times mrp_render_device on 4096 lanes of MultiRobotPuzzle-v0 at 160x120 (HIP events)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gym_puzzles_amd import Batch

env_id = int(sys.argv[1]) if len(sys.argv) > 1 else 0
n, W, H = 4096, 160, 120
b = Batch(env_id, n, seed=1)
b.reset()
for _ in range(10):
    b.step()
lanes = torch.arange(n, dtype=torch.int32, device="cuda")
img = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda")
b.set_stream(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
for _ in range(3):
    b.render_device(lanes.data_ptr(), n, W, H, img.data_ptr())
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
K = 20
e0.record()
for _ in range(K):
    b.render_device(lanes.data_ptr(), n, W, H, img.data_ptr())
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
print(json.dumps({"env_id": env_id, "lanes": n, "width": W, "height": H, "ms_per_batch": ms,
                  "frames_per_s": n / ms * 1e3, "out_GB_per_s": n * W * H * 3 / ms / 1e6,
                  "nonzero_frac": float((img != 0).float().mean())}))
