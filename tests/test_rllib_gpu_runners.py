"""Env runners acting on GPU shares (``num_gpus_per_env_runner``) with the learner's
weights broadcast over HIP IPC handles (BASELINE config 4 hand-off): runner modules
live on the GPU, and after a sync they hold exactly the learner's weights."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_ppo_gpu_runners_ipc_weights():
    import cluster_anywhere_amd as ray
    from cluster_anywhere_amd import rllib
    from cluster_anywhere_amd.core import api as core

    ray.init(num_cpus=4, num_gpus=1)
    try:
        cfg = (rllib.PPOConfig().environment("FakeAtari-v0")
               .env_runners(num_env_runners=2, num_envs_per_env_runner=2, num_gpus_per_env_runner=0.1,
                            rollout_fragment_length=32)
               .learners(num_learners=0, num_gpus_per_learner=1)
               .training(train_batch_size=128, minibatch_size=64, num_epochs=1).debugging(seed=0))
        algo = cfg.build()
        assert algo._ipc_weights()
        for _ in range(2):
            r = algo.train()
        assert r["num_env_steps_sampled_lifetime"] >= 256
        algo._sync_weights()
        want = algo.learner_group.get_module_state()
        for st in core.get([w.get_weights.remote() for w in algo.env_runner_group.remote]):
            for k, v in want.items():
                assert torch.equal(st[k], v), k
        dev = core.get(algo.env_runner_group.remote[0].__ray_call__.remote(lambda self: str(self.device)))
        assert dev.startswith("cuda")
        algo.stop()
    finally:
        ray.shutdown()


def test_restarted_gpu_runner_gets_the_synced_weights():
    """a runner recreated after an IPC weight broadcast is caught up
    from the SAME ref; the device snapshot behind its HIP IPC handles must still be
    alive then. Kill a runner, churn the driver's caching allocator (free the learner's
    old snapshot, allocate over it), restore, and compare weights bit for bit."""
    import os
    import signal

    import cluster_anywhere_amd as ray
    from cluster_anywhere_amd import rllib
    from cluster_anywhere_amd.core import api as core

    ray.init(num_cpus=4, num_gpus=1)
    try:
        cfg = (rllib.PPOConfig().environment("FakeAtari-v0")
               .env_runners(num_env_runners=2, num_envs_per_env_runner=2, num_gpus_per_env_runner=0.1,
                            rollout_fragment_length=32)
               .learners(num_learners=0, num_gpus_per_learner=1)
               .training(train_batch_size=128, minibatch_size=64, num_epochs=1).debugging(seed=0))
        algo = cfg.build()
        assert algo._ipc_weights()
        algo.train()
        algo._sync_weights()
        want = {k: v.clone() for k, v in algo.learner_group.get_module_state().items()}
        grp = algo.env_runner_group
        pid = core.get(grp.remote[1].__ray_call__.remote(lambda self: os.getpid()))
        os.kill(pid, signal.SIGKILL)
        # churn: blocks the allocator freed would be reused by these
        junk = [torch.randn(1 << 20, device="cuda") for _ in range(64)]
        del junk
        torch.cuda.synchronize()
        grp.healthy[1] = False
        assert grp.restore([1]) == [1]
        st = core.get(grp.remote[1].get_weights.remote())
        for k, v in want.items():
            assert torch.equal(st[k].to(v.device), v), k
        algo.stop()
    finally:
        ray.shutdown()
