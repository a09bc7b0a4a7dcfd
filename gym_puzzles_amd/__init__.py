"""gym_puzzles_amd -- MI355X-native MultiRobotPuzzle step (HIP/gfx950) behind the
gym_puzzles env interface.  See DESIGN.md.

    Batch                  N lanes on one GPU, thin wrapper of the C ABI (include/mrp.h)
    envs.MultiRobotPuzzle  gym-style single env classes (same names as gym_puzzles.envs)
    envs.make(id)          gym.make equivalent (adds gym 0.21's TimeLimit)
    MultiRobotPuzzleVecEnv SB3-style vectorised env with on-device auto-reset
    MultiRobotPuzzleVecNormalize / DeviceVecNormalize
                           SB3 VecNormalize + Monitor statistics on the device
"""
from ._native import ENV_IDS, Batch, MrpError, env_dims  # noqa: F401


def __getattr__(name):
    # the env classes import lazily so that `import gym_puzzles_amd` never touches the GPU
    if name in ("MultiRobotPuzzle", "MultiRobotPuzzleHeavy", "MultiRobotPuzzle2", "MultiRobotPuzzleHeavy2",
                "MultiRobotPuzzleHeavy2ThreeBlock", "RobotPuzzleBase", "make"):
        from . import envs
        return getattr(envs, name)
    if name in ("MultiRobotPuzzleVecEnv", "MultiRobotPuzzleVecNormalize", "DeviceVecNormalize"):
        from . import vec_env
        return getattr(vec_env, name)
    raise AttributeError(name)
