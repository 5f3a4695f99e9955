"""Tune callbacks and loggers (reference: python/ray/tune/callback.py,
logger/json.py, logger/csv.py, progress_reporter.py)."""
from __future__ import annotations

import csv
import json
import os
import sys
import time


class Callback:
    def on_trial_start(self, iteration, trials, trial, **info):
        pass

    def on_trial_result(self, iteration, trials, trial, result, **info):
        pass

    def on_trial_complete(self, iteration, trials, trial, **info):
        pass

    def on_trial_error(self, iteration, trials, trial, **info):
        pass

    def on_experiment_end(self, trials, **info):
        pass


class LoggerCallback(Callback):
    def log_trial_result(self, iteration, trial, result):
        pass

    def on_trial_result(self, iteration, trials, trial, result, **info):
        self.log_trial_result(iteration, trial, result)


class JsonLoggerCallback(LoggerCallback):
    """Extra JSON log (the controller already writes result.json per trial)."""

    def __init__(self, filename: str = "result_extra.json"):
        self.filename = filename

    def log_trial_result(self, iteration, trial, result):
        with open(os.path.join(trial.local_path, self.filename), "a") as f:
            f.write(json.dumps(result, default=str) + "\n")


class CSVLoggerCallback(LoggerCallback):
    def __init__(self, filename: str = "progress_extra.csv"):
        self.filename = filename
        self.keys = {}

    def log_trial_result(self, iteration, trial, result):
        row = {k: v for k, v in result.items() if not isinstance(v, (dict, list))}
        p = os.path.join(trial.local_path, self.filename)
        new = trial.trial_id not in self.keys
        if new:
            self.keys[trial.trial_id] = list(row)
        with open(p, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=self.keys[trial.trial_id], extrasaction="ignore")
            if new:
                w.writeheader()
            w.writerow(row)


class CLIReporter(Callback):
    """Prints a trial table at most every ``max_report_frequency`` seconds."""

    def __init__(self, metric_columns=None, parameter_columns=None, max_report_frequency: float = 5.0,
                 out=None):
        self.metric_columns = metric_columns
        self.parameter_columns = parameter_columns
        self.freq = max_report_frequency
        self.last = 0.0
        self.out = out or sys.stdout

    def _table(self, trials):
        lines = [f"== Status: {sum(t.status == 'RUNNING' for t in trials)} running, "
                 f"{sum(t.status == 'TERMINATED' for t in trials)} terminated, "
                 f"{sum(t.status == 'ERROR' for t in trials)} errored =="]
        for t in trials:
            m = t.last_result
            cols = self.metric_columns or [k for k in m if isinstance(m.get(k), (int, float))][:4]
            ps = self.parameter_columns or list(t.config)[:4]
            lines.append(f"{t.trial_name:<32} {t.status:<10} "
                         + " ".join(f"{p}={t.config.get(p)}" for p in ps) + " | "
                         + " ".join(f"{c}={m.get(c)}" for c in cols))
        return "\n".join(lines)

    def on_trial_result(self, iteration, trials, trial, result, **info):
        if time.time() - self.last >= self.freq:
            self.last = time.time()
            print(self._table(trials), file=self.out)

    def on_experiment_end(self, trials, **info):
        print(self._table(trials), file=self.out)


ProgressReporter = CLIReporter
