"""bppo — MI355X-native rollout -> GAE -> PPO-update hot path of burn-ppo.

Host mirror of the reference's surfaces over libbppo.so (include/bppo.h)."""
from ._lib import BppoError, lib  # noqa: F401
from .host import make_config, minibatch_sizes, orthogonal_init, schedule_get  # noqa: F401
from .ppo import (ActorCritic, Context, RolloutBuffer, Trainer, VecEnv, collect_rollouts,  # noqa: F401
                  compute_gae, perf_scalars, ppo_update, rollout_episodes, train_step)
