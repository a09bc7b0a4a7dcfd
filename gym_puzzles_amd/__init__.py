"""gym_puzzles_amd -- MI355X-native MultiRobotPuzzle step (HIP/gfx950) behind the
gym_puzzles env interface.  See DESIGN.md."""
from ._native import ENV_IDS, Batch, MrpError, env_dims  # noqa: F401
