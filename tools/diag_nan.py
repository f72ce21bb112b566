import torch, numpy as np, sys
sys.path.insert(0, ".")
from tum_adlr_deep_reinforcement_learning_amd.replay import OffPolicyCollector, ReplayBuffer
from tum_adlr_deep_reinforcement_learning_amd.vec_env import FixedWingVecEnv
n, steps = 512, 12
env = FixedWingVecEnv(n, config_kw={"steps_max": 8}, sim_config_kw={"turbulence": False}, device="cuda:0", seed=3, return_tensors=True)
print(env.obs_names() if hasattr(env, "obs_names") else "")
buf = ReplayBuffer(n * 16, env.observation_space, env.action_space, device="cuda:0", n_envs=n)
col = OffPolicyCollector(env, buf, learning_starts=10 ** 9, seed=1)
col.collect(steps)
obs = buf.observations[:steps].cpu(); nxt = buf.next_observations[:steps].cpu(); d = buf.dones[:steps].cpu()
print("nan obs per step", torch.isnan(obs).any(-1).sum(-1).tolist())
print("nan cols", torch.isnan(obs).any(0).any(0).nonzero().ravel().tolist())
print("nan next per step", torch.isnan(nxt).any(-1).sum(-1).tolist())
print("dones per step", d.sum(-1).tolist())
i = torch.isnan(obs).any(-1).nonzero()[:3]
print(i)
for s, e in i.tolist():
    print(s, e, obs[s, e].tolist(), buf.actions[s, e].tolist())
print("act range", env.action_space.low, env.action_space.high)
