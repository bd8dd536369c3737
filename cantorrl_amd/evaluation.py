"""Episode statistics of the reference evaluation loops, from device episode records.

`he_rollout_policy` (HedgingVecEnv.rollout_policy / evaluate_policy) appends one
he_episode_record per finished episode on the device; these functions reduce the
(small) record arrays exactly as the reference scripts reduce their python lists:

* `baseline_statistics`  -- evaluate_baseline_policy, src/agents/baselines.py:56-72:
  per episode sum(raw_pnl_deviation_abs)/steps and sum(transaction_costs_total)/steps,
  then mean / mean / std over episodes.
* `train_eval_statistics` -- train_ppo_v2.py:515-531: per episode
  |sum(per_share_step_pnl)| / episode_length and sum(costs) / episode_length, then
  mean, mean, std and CVaR95 (mean of the sorted top 5 %).
"""
import numpy as np


def baseline_statistics(records):
    r = np.asarray(records)
    if r.size == 0:
        return dict(mean_abs_pnl=0, mean_cost=0, std_abs_pnl=0)
    steps = r["length"].astype(np.float64)
    ep_abs = r["abs_pnl_sum"] / steps
    ep_cost = r["cost_sum"] / steps
    return dict(mean_abs_pnl=float(np.mean(ep_abs)), mean_cost=float(np.mean(ep_cost)),
                std_abs_pnl=float(np.std(ep_abs)))


def train_eval_statistics(records, episode_length):
    r = np.asarray(records)
    if r.size == 0:
        return dict(mean_abs_pnl=0, mean_cost=0, std_abs_pnl=0, cvar95_abs_pnl=0.0)
    ep_abs = [abs(x) / episode_length for x in r["per_share_pnl_sum"]]
    ep_cost = [c / episode_length for c in r["cost_sum"]]
    srt = sorted(ep_abs)
    return dict(mean_abs_pnl=float(np.mean(ep_abs)), mean_cost=float(np.mean(ep_cost)),
                std_abs_pnl=float(np.std(ep_abs)), cvar95_abs_pnl=float(np.mean(srt[int(0.95 * len(srt)):])))
