"""Host-side pieces of the reference's interface that are plain arithmetic:
config presets (configs/*.toml), minibatch split (ppo.rs:1820-1831), the
learning-rate schedule (schedule.rs:54-78), orthogonal init (mlp.rs:16-38)."""
import numpy as np

from . import _lib as L
from .dist import shard


def minibatch_sizes(batch_size, num_minibatches):
    """ppo.rs:1820-1831: base = B / M, the first B % M minibatches get +1; empty ones skipped."""
    base, rem = divmod(batch_size, num_minibatches)
    return [base + (1 if i < rem else 0) for i in range(num_minibatches)
            if base + (1 if i < rem else 0) > 0]


def shaping_schedule(c):
    """reward_shaping_coef as (value, step) milestones: a number is Schedule::constant
    (schedule.rs:44-46, 232-251), a list is sorted by step (schedule.rs:257-270)."""
    v = c["reward_shaping_coef"]
    if isinstance(v, (int, float)):
        return [(float(v), 0)]
    return sorted(((float(a), int(b)) for a, b in v), key=lambda p: p[1])


def schedule_get(points, step):
    """schedule.rs:54-78 piecewise-linear [(value, step), ...]."""
    if not points:
        return 0.0
    if len(points) == 1 or step <= points[0][1]:
        return float(points[0][0])
    for (v1, s1), (v2, s2) in zip(points, points[1:]):
        if s1 <= step < s2:
            return v1 + (v2 - v1) * ((step - s1) / (s2 - s1))
    return float(points[-1][0])


# Environment constants: OBSERVATION_DIM, ACTION_COUNT, NUM_PLAYERS, PRIVILEGED_OBS_DIM
# (cartpole.rs, connect_four.rs, liars_dice.rs:455-460, skull.rs:1046-1060)
ENV_DIMS = {"cartpole": (5, 2, 1, 0), "connect_four": (86, 7, 2, 0), "liars_dice": (270, 49, 4, 120),
            "skull": (135, 33, 6, 200)}

# config presets = the reference's configs + BASELINE.json sizes (SURVEY.md CfgA..CfgE)
BASE = dict(env="cartpole", num_envs=32, num_steps=128, hidden_size=64, num_hidden=2, activation="relu",
            network_type="mlp", critic_hidden_size=None, critic_num_hidden=None, num_epochs=4,
            num_minibatches=4, normalize_obs=False, normalize_returns=None, clip_value=False, gamma=0.99,
            gae_lambda=0.95, clip_epsilon=0.2, value_coef=0.5, max_grad_norm=0.5, adam_epsilon=1e-5,
            target_kl=None, return_clip=10.0, reward_shaping_coef=0.0, learning_rate=[(2.5e-4, 0)],
            entropy_coef=[(0.01, 0)], seed=42, player_count=4, split_networks=False, shuffle_windows=False,
            # network_type = "cnn" (config.rs:996-1010 defaults)
            num_conv_layers=2, conv_channels=[8, 8], kernel_size=3, cnn_fc_hidden_size=32, cnn_num_fc_layers=1)

PRESETS = {
    # configs/test.toml (CfgA runs it with --num-envs 8 --num-steps 128)
    "test": dict(num_envs=2, num_steps=8, num_epochs=1, num_minibatches=1, hidden_size=16, num_hidden=1,
                 learning_rate=[(1e-3, 0)]),
    # configs/cartpole.toml (CfgB: num_envs 65536)
    "cartpole": dict(num_envs=32, learning_rate=[(1e-3, 0)], entropy_coef=[(0.01, 0)], normalize_obs=True,
                     num_epochs=4, hidden_size=64, num_hidden=2),
    # configs/connect_four.toml (CfgC: num_envs 16384, pool off)
    "connect_four": dict(env="connect_four", num_envs=128, num_steps=64,
                         learning_rate=[(1e-3, 0), (1e-4, 40_000_000)], clip_epsilon=0.1,
                         entropy_coef=[(0.05, 0)], target_kl=0.02, num_epochs=6, hidden_size=512),
    # configs/liars_dice_ctde.toml (CfgD: num_envs 32768, pool off)
    "liars_dice_ctde": dict(env="liars_dice", num_envs=256, network_type="ctde", hidden_size=256,
                            critic_hidden_size=512, critic_num_hidden=3, reward_shaping_coef=0.05,
                            learning_rate=[(3e-4, 0)], gamma=0.97, gae_lambda=0.90,
                            entropy_coef=[(0.05, 0)], value_coef=1.0, target_kl=0.025, num_epochs=4,
                            num_minibatches=8),
    # configs/skull.toml / skull_ctde.toml ([player_count] Fixed 4)
    "skull": dict(env="skull", num_envs=128, num_steps=128, hidden_size=256, num_hidden=3,
                  learning_rate=[(1e-3, 0), (3e-4, 80_000_000), (0.0, 100_000_000)], gamma=0.99, gae_lambda=0.9,
                  clip_epsilon=0.1, entropy_coef=[(0.05, 0)], value_coef=0.5, target_kl=0.02, num_epochs=4,
                  num_minibatches=8),
    "skull_ctde": dict(env="skull", num_envs=128, num_steps=128, network_type="ctde", hidden_size=256,
                       num_hidden=3, critic_hidden_size=256, critic_num_hidden=3,
                       learning_rate=[(1e-3, 0), (3e-4, 80_000_000), (0.0, 100_000_000)], gamma=0.99,
                       gae_lambda=0.9, clip_epsilon=0.1, entropy_coef=[(0.05, 0)], value_coef=0.5, target_kl=0.02,
                       num_epochs=4, num_minibatches=8),
}


def make_config(preset="cartpole", **over):
    c = dict(BASE)
    c.update(PRESETS[preset])
    c.update(over)
    return c


def num_players(env):
    return ENV_DIMS[env][2]


def to_struct(c, rank=0, world=1, envs_per_rank=None):
    n = envs_per_rank if envs_per_rank is not None else c["num_envs"]
    nr = c["normalize_returns"]
    if nr is None:
        nr = num_players(c["env"]) == 1          # main.rs:243
    s = L.Config()
    s.env_kind = L.ENV_KINDS[c["env"]]
    s.num_envs = n
    s.num_steps = c["num_steps"]
    s.hidden_size = c["hidden_size"]
    s.num_hidden = c["num_hidden"]
    s.relu = int(c["activation"] == "relu")
    s.ctde = int(c["network_type"] == "ctde")
    s.critic_hidden_size = c["critic_hidden_size"] or c["hidden_size"]
    s.critic_num_hidden = c["critic_num_hidden"] or c["num_hidden"]
    s.num_epochs = c["num_epochs"]
    s.num_minibatches = c["num_minibatches"]
    s.normalize_obs = int(c["normalize_obs"])
    s.normalize_returns = int(nr)
    s.clip_value = int(c["clip_value"])
    for k in ("gamma", "gae_lambda", "clip_epsilon", "value_coef", "max_grad_norm", "adam_epsilon",
              "return_clip"):
        setattr(s, k, float(c[k]))
    # a Schedule's initial value; the milestones follow via bppo_set_reward_shaping_schedule
    s.reward_shaping_coef = schedule_get(shaping_schedule(c), 0)
    s.target_kl = -1.0 if c["target_kl"] is None else float(c["target_kl"])
    s.seed = c["seed"]
    s.normalize_values = int(bool(c.get("normalize_values", False)))
    s.player_count = int(c.get("player_count", 4)) if c["env"] == "skull" else 0
    s.split_networks = int(bool(c.get("split_networks", False)))
    s.shuffle_windows = int(bool(c.get("shuffle_windows", False)))
    s.cnn = int(c["network_type"] == "cnn")
    if s.cnn:
        s.num_conv_layers = c["num_conv_layers"]
        ch = conv_channels(c)
        for i in range(4):
            s.conv_channels[i] = ch[min(i, len(ch) - 1)]
        s.kernel_size = c["kernel_size"]
        s.cnn_fc_hidden_size = c["cnn_fc_hidden_size"]
        s.cnn_num_fc_layers = c["cnn_num_fc_layers"]
    # W > 1: global env index = rank * n + i; main RNG stream = rank
    s.env_seed_base, s.rng_stream = shard(c, rank, world, n)
    return s


def conv_channels(c):
    """cnn.rs:84-90: channels of conv layer i, the last entry repeated"""
    ch = list(c["conv_channels"])
    if not ch:
        raise ValueError("conv_channels must not be empty")          # config.rs:1575-1577
    return [ch[min(i, len(ch) - 1)] for i in range(c["num_conv_layers"])]


def layer_shapes(c):
    """Burn record order: hidden..., policy head, value head (MLP) /
    actor hidden..., critic hidden..., policy, value (MLP with split_networks, mlp.rs:47-62) /
    actor hidden..., policy, critic hidden..., value (CTDE) /
    conv layers (as (Cin*k*k, Cout)), FC layers, policy, value (CNN)."""
    obs, act, _, priv = ENV_DIMS[c["env"]]
    shapes, gains = [], []
    hg = np.sqrt(2.0) if c["activation"] == "relu" else 1.0
    i = obs
    if c["network_type"] == "cnn":
        if c["env"] != "connect_four":
            raise ValueError("CNN requires OBSERVATION_SHAPE")          # cnn.rs:73-74
        H, W, C0 = 6, 7, 2                                              # connect_four.rs:217
        cin = C0
        for co in conv_channels(c):
            shapes.append((cin * c["kernel_size"] ** 2, co)); gains.append(None); cin = co
        i = H * W * cin + (obs - H * W * C0)
        for _ in range(c["cnn_num_fc_layers"]):
            shapes.append((i, c["cnn_fc_hidden_size"])); gains.append(hg); i = c["cnn_fc_hidden_size"]
        if c.get("split_networks"):        # cnn.rs:116-135: the critic's own conv stack and FC layers
            n_trunk = len(shapes)
            shapes += shapes[:n_trunk]; gains += gains[:n_trunk]
        shapes.append((i, act)); gains.append(0.01)
        shapes.append((i, 1)); gains.append(1.0)
        return shapes, gains
    for _ in range(c["num_hidden"]):
        shapes.append((i, c["hidden_size"])); gains.append(hg); i = c["hidden_size"]
    if c.get("split_networks") and c["network_type"] == "mlp":
        ci = obs                                                     # mlp.rs:100-114: critic trunk on obs
        for _ in range(c["num_hidden"]):
            shapes.append((ci, c["hidden_size"])); gains.append(hg); ci = c["hidden_size"]
        shapes.append((i, act)); gains.append(0.01)
        shapes.append((ci, 1)); gains.append(1.0)
        return shapes, gains
    shapes.append((i, act)); gains.append(0.01)
    if c["network_type"] == "ctde":
        ci = priv + obs
        for _ in range(c["critic_num_hidden"] or c["num_hidden"]):
            w = c["critic_hidden_size"] or c["hidden_size"]
            shapes.append((ci, w)); gains.append(hg); ci = w
        shapes.append((ci, 1)); gains.append(1.0)
    else:
        shapes.append((i, 1)); gains.append(1.0)
    return shapes, gains


def orthogonal_init(c, seed=0):
    """mlp.rs:16-38 / ctde.rs:64-123: orthogonal weights with gains sqrt(2)|1 (hidden),
    0.01 (policy), 1.0 (value); zero biases.  Burn's init RNG is not reproducible
    here, so parity runs load these weights into both the oracle and the device."""
    rng = np.random.default_rng(seed)
    out = []
    shapes, gains = layer_shapes(c)
    for (i, o), g in zip(shapes, gains):
        if g is None:
            # Conv2d (Burn default KaimingUniform, gain 1/sqrt(3)): U(-1/sqrt(fan_in), 1/sqrt(fan_in))
            # for the weight [Cout][Cin][k][k] and the bias
            bound = 1.0 / np.sqrt(i)
            out.append(rng.uniform(-bound, bound, o * i).astype(np.float32))
            out.append(rng.uniform(-bound, bound, o).astype(np.float32))
            continue
        a = rng.standard_normal((max(i, o), min(i, o)))
        q, r = np.linalg.qr(a)
        q = q * np.sign(np.diag(r))
        w = q if i >= o else q.T
        out.append((g * w).astype(np.float32).reshape(-1))
        out.append(np.zeros(o, np.float32))
    return np.concatenate(out)
