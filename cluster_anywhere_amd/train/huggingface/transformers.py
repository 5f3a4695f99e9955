"""Run a ``transformers.Trainer`` inside ``TorchTrainer`` workers (reference:
python/ray/train/huggingface/transformers/_transformers_utils.py:30
``RayTrainReportCallback`` and :104 ``prepare_trainer``).

* :class:`RayTrainReportCallback` turns every HF checkpoint save into a
  ``train.report(metrics, checkpoint=...)`` (the checkpoint directory HF just
  wrote, so Train's top-k retention and ``Result.checkpoint`` work unchanged);
  rank 0's metrics are the merged HF logs since the last save.
* :func:`prepare_trainer` makes the Trainer consume Ray Data shards
  (``train.get_dataset_shard``): a ``DataIterator`` / ``Dataset`` train or eval
  dataset is wrapped in a torch ``IterableDataset`` that streams rows, and the
  HF data loaders are rebuilt without a sampler (the shard is already this
  rank's part). Process-group setup is Train's (RCCL on MI355X, gloo on CPU):
  HF's ``TrainingArguments`` picks it up from the initialised default group.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from typing import Any, Dict

import transformers
from transformers.trainer_callback import TrainerCallback

CHECKPOINT_NAME = "checkpoint"


class RayTrainReportCallback(TrainerCallback):
    """Report HF logs and checkpoints to Train on every save."""

    def __init__(self):
        super().__init__()
        self._metrics: Dict[str, Any] = {}

    def on_log(self, args, state, control, model=None, logs=None, **kwargs):
        if logs:
            self._metrics.update({k: v for k, v in logs.items() if isinstance(v, (int, float))})

    def on_save(self, args, state, control, **kwargs):
        from ... import train
        from ..checkpoint import Checkpoint

        src = os.path.join(args.output_dir, f"checkpoint-{state.global_step}")
        metrics = dict(self._metrics, step=state.global_step, epoch=state.epoch)
        with tempfile.TemporaryDirectory() as tmp:
            ckpt = None
            if os.path.isdir(src):
                dst = os.path.join(tmp, CHECKPOINT_NAME)
                shutil.copytree(src, dst)
                ckpt = Checkpoint.from_directory(dst)
            train.report(metrics, checkpoint=ckpt)
        self._metrics = {}


def _iterable(ds, batch_size=None):
    import torch

    class _Rows(torch.utils.data.IterableDataset):
        def __iter__(self):
            it = ds.iter_rows() if hasattr(ds, "iter_rows") else iter(ds)
            for row in it:
                yield {k: (torch.tensor(v) if not isinstance(v, (str, bytes)) else v) for k, v in row.items()}

    return _Rows()


def prepare_trainer(trainer: "transformers.Trainer") -> "transformers.Trainer":
    """Wire a ``transformers.Trainer`` to Ray Data shards (see module docstring)."""
    import torch

    def _is_ray(ds):
        mod = type(ds).__module__
        return ds is not None and mod.startswith("cluster_anywhere_amd.data")

    if _is_ray(getattr(trainer, "train_dataset", None)):
        trainer.train_dataset = _iterable(trainer.train_dataset)
    if _is_ray(getattr(trainer, "eval_dataset", None)):
        trainer.eval_dataset = _iterable(trainer.eval_dataset)

    base_train = trainer.get_train_dataloader
    base_eval = trainer.get_eval_dataloader

    def get_train_dataloader():
        ds = trainer.train_dataset
        if isinstance(ds, torch.utils.data.IterableDataset):
            return torch.utils.data.DataLoader(ds, batch_size=trainer.args.per_device_train_batch_size,
                                               collate_fn=trainer.data_collator)
        return base_train()

    def get_eval_dataloader(eval_dataset=None):
        ds = eval_dataset if eval_dataset is not None else trainer.eval_dataset
        if isinstance(ds, torch.utils.data.IterableDataset):
            return torch.utils.data.DataLoader(ds, batch_size=trainer.args.per_device_eval_batch_size,
                                               collate_fn=trainer.data_collator)
        return base_eval(eval_dataset)

    trainer.get_train_dataloader = get_train_dataloader
    trainer.get_eval_dataloader = get_eval_dataloader
    return trainer


__all__ = ["RayTrainReportCallback", "prepare_trainer"]
