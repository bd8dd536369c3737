"""CPU restatement of Stable-Baselines3 2.6.0 VecNormalize / RunningMeanStd / Monitor
episode sums, as the reference uses them (train_ppo_v2.py:119, :204, :305, :450-453).

TEST INFRASTRUCTURE ONLY: the checker for cantorrl_amd.vec_normalize (HIP kernels in
cantorrl_amd/csrc/vecnorm.hip).  SB3 is not installed in this image and its source is
not under /root/reference, so this follows SB3 2.6.0's published algorithm
(stable_baselines3/common/running_mean_std.py, vec_env/vec_normalize.py,
monitor.py): parity with SB3 itself is unpinned.

moments="sb3" reproduces SB3's NumPy calls literally -- np.mean / np.var over axis 0
of the f32 observation batch accumulate in f32; moments="f64" takes the batch moments
in f64 (what the device computes), the tight reference for the kernels.
"""
import numpy as np


class RunningMeanStd:
    def __init__(self, epsilon=1e-4, shape=(), moments="sb3"):
        self.mean = np.zeros(shape, np.float64)
        self.var = np.ones(shape, np.float64)
        self.count = epsilon
        self.moments = moments

    def update(self, arr):
        if self.moments == "f64":
            arr = np.asarray(arr, np.float64)
        batch_mean = np.mean(arr, axis=0)
        batch_var = np.var(arr, axis=0)
        self.update_from_moments(batch_mean, batch_var, arr.shape[0])

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        delta = batch_mean - self.mean
        tot_count = self.count + batch_count
        new_mean = self.mean + delta * batch_count / tot_count
        m_a = self.var * self.count
        m_b = batch_var * batch_count
        m_2 = m_a + m_b + np.square(delta) * self.count * batch_count / tot_count
        self.mean = new_mean
        self.var = m_2 / tot_count
        self.count = batch_count + self.count


class VecNormalizeOracle:
    """VecNormalize over externally stepped batches: reset(obs) / step(obs, rewards,
    dones, terminal_obs) mirror VecNormalize.reset / step_wait."""

    def __init__(self, num_envs, obs_dim=13, training=True, norm_obs=True, norm_reward=True, clip_obs=10.0,
                 clip_reward=10.0, gamma=0.99, epsilon=1e-8, moments="sb3"):
        self.obs_rms = RunningMeanStd(shape=(obs_dim,), moments=moments)
        self.ret_rms = RunningMeanStd(shape=(), moments=moments)
        self.training, self.norm_obs, self.norm_reward = training, norm_obs, norm_reward
        self.clip_obs, self.clip_reward, self.gamma, self.epsilon = clip_obs, clip_reward, gamma, epsilon
        self.returns = np.zeros(num_envs)
        self.ep_ret = np.zeros(num_envs)
        self.ep_len = np.zeros(num_envs, np.int64)

    def _normalize_obs(self, obs):
        return np.clip((obs - self.obs_rms.mean) / np.sqrt(self.obs_rms.var + self.epsilon), -self.clip_obs,
                       self.clip_obs)

    def normalize_obs(self, obs):
        return self._normalize_obs(obs).astype(np.float32) if self.norm_obs else obs.copy()

    def normalize_reward(self, reward):
        if self.norm_reward:
            return np.clip(reward / np.sqrt(self.ret_rms.var + self.epsilon), -self.clip_reward, self.clip_reward)
        return reward

    def reset(self, obs):
        self.returns = np.zeros_like(self.returns)
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        return self.normalize_obs(obs)

    def step(self, obs, rewards, dones, terminal_obs=None, env_rewards=None):
        """-> (obs, rewards, terminal_obs of done rows, {i: (ep_return, ep_length)}).

        rewards: the VecEnv's reward buffer (what VecNormalize sees); env_rewards: the envs'
        own f64 step rewards, which Monitor sums -- Monitor wraps each env inside the VecEnv
        (train_ppo_v2.py:119; monitor.py appends float(reward) of the env's step,
        hedging_env_v2.py:262,294).  env_rewards=None sums `rewards` (an env whose reward is
        already that buffer's dtype)."""
        if self.training and self.norm_obs:
            self.obs_rms.update(obs)
        obs_n = self.normalize_obs(obs)
        if self.training:
            self.returns = self.returns * self.gamma + rewards
            self.ret_rms.update(self.returns)
        rew_n = self.normalize_reward(rewards)
        tobs_n = None
        if terminal_obs is not None:
            tobs_n = {int(i): self.normalize_obs(terminal_obs[i]) for i in np.nonzero(dones)[0]}
        self.returns[dones] = 0
        # Monitor: sum / count of the envs' own (f64) rewards per episode, in step order
        self.ep_ret += np.asarray(rewards if env_rewards is None else env_rewards, np.float64)
        self.ep_len += 1
        eps = {int(i): (self.ep_ret[i], int(self.ep_len[i])) for i in np.nonzero(dones)[0]}
        self.ep_ret[dones] = 0.0
        self.ep_len[dones] = 0
        return obs_n, rew_n, tobs_n, eps
