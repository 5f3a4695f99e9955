"""GTrXL attention core in the default RLModule (reference: RLlib attention nets,
``use_attention``; rllib/examples/attention_net.py on memory tasks)."""
import torch

from cluster_anywhere_amd import rllib
from cluster_anywhere_amd.rllib.algorithms.algorithm import concat_fragments
from cluster_anywhere_amd.rllib.core.rl_module import GTrXLCore


def _cfg(**kw):
    return (rllib.PPOConfig().environment("RepeatAfterMe-v0")
            .env_runners(num_envs_per_env_runner=16, rollout_fragment_length=40)
            .training(lr=3e-3, train_batch_size=640, minibatch_size=160, num_epochs=6, gamma=0.5, lambda_=0.9,
                      vf_loss_coeff=0.5,
                      model={"fcnet_hiddens": [64], "use_attention": True, "attention_dim": 32,
                             "attention_num_heads": 2, "attention_num_transformer_units": 1,
                             "attention_memory_inference": 4, "max_seq_len": 20, **kw})
            .reporting(metrics_num_episodes_for_smoothing=32).debugging(seed=0))


def test_gtrxl_memory_is_a_sliding_window():
    torch.manual_seed(0)
    core = GTrXLCore(3, dim=8, heads=2, units=2, memory=3, mlp_dim=8)
    mem = torch.zeros(2, core.state_size)
    xs = [torch.randn(2, 3) for _ in range(5)]
    for x in xs:
        y, mem = core.step(x, mem)
    assert y.shape == (2, 8) and mem.shape == (2, 2 * 3 * 8)
    # unit 0's memory holds the projected inputs of the last 3 steps, oldest first
    m0 = mem.view(2, 2, 3, 8)[:, 0]
    assert torch.allclose(m0[:, -1], core.inp(xs[-1]), atol=1e-6)
    assert torch.allclose(m0[:, 0], core.inp(xs[-3]), atol=1e-6)


def test_attention_sequences_reproduce_sampled_outputs():
    algo = _cfg().env_runners(num_envs_per_env_runner=4).build()
    lrn = algo.learner_group.local
    frag = concat_fragments(algo.env_runner_group.sample())
    assert frag["state_in_mem"].shape == (40, 4, 4 * 32) and frag["last_state_mem"].shape == (4, 4 * 32)
    b = lrn.postprocess(frag)
    assert b["obs"].shape == (8, 20, 2) and b["state_in_mem"].shape == (8, 4 * 32)
    st = {k[len("state_in_"):]: v for k, v in b.items() if k.startswith("state_in_")}
    out = lrn.module.forward_train(dict(b, state_in=st))
    assert torch.allclose(out["action_dist_inputs"], b["action_dist_inputs"].reshape(-1, 2), atol=1e-4)
    algo.stop()


def test_attention_ppo_learns_memory_task():
    algo = _cfg().build()
    best = 0.0
    for _ in range(20):
        best = max(best, algo.train()["env_runners"]["episode_return_mean"])
        if best > 17:
            break
    assert best > 15, best  # chance ~9.5, optimum 19
    algo.stop()
