"""Where the gym-style single env's step time goes (diagnostic, GPU box):
    python tools/single_env_timing.py [ENV_NAME] [STEPS]
Times, per step of one lane: the k_step kernel alone (HIP events on the ctx's stream, device
inputs), the host-pointer ABI call (mrp_step_ex through Batch.step: zero-copy pinned I/O, one
synchronisation), and the gym-style env.step() (TimeLimit wrapper, float64 obs, info)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch

    from gym_puzzles_amd import Batch, make
    name = sys.argv[1] if len(sys.argv) > 1 else "MultiRobotPuzzle-v0"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    env = make(name)
    env.reset()
    eid = env.unwrapped.env_id
    A = env.action_space.shape[0]
    acts = np.random.RandomState(0).uniform(-1, 1, size=(steps + 20, A)).astype(np.float32)
    res = {"env": name}
    # gym-style env.step
    for k in range(20):
        if env.step(acts[k])[2]:
            env.reset()
    t0 = time.perf_counter()
    for k in range(steps):
        if env.step(acts[20 + k])[2]:
            env.reset()
    res["env_step_us"] = (time.perf_counter() - t0) / steps * 1e6
    # Batch.step (the C ABI's host-pointer step)
    b = Batch(eid, 1, seed=3)
    b.set_auto_reset(True)
    b.reset()
    for k in range(20):
        b.step(acts[k][None])
    t0 = time.perf_counter()
    for k in range(steps):
        b.step(acts[20 + k][None])
    res["batch_step_us"] = (time.perf_counter() - t0) / steps * 1e6
    # the kernel alone: device-RNG actions, device outputs, events on the ctx's stream
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    b.set_stream(s.cuda_stream)
    obs = torch.zeros((1, b.obs_dim), device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(20):
        b.step_device(0, obs.data_ptr())
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(steps):
        b.step_device(0, obs.data_ptr())
    e1.record(s)
    torch.cuda.synchronize()
    res["kernel_stream_us"] = e0.elapsed_time(e1) * 1e3 / steps
    t0 = time.perf_counter()
    for _ in range(steps):
        b.step_device(0, obs.data_ptr())
        b.synchronize()
    res["launch_sync_us"] = (time.perf_counter() - t0) / steps * 1e6
    b.close()
    env.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
