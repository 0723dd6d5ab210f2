"""Minimal logger with the reference's dict-of-lists layout (``sac_eo/common/logger.py``);
checkpoints are written as JSON + NumPy .npz (no pickle)."""
import json
import os

import numpy as np


class Logger:
    def __init__(self):
        self.param_dict = {}
        self.train_dict = {}
        self.eval_dict = {}
        self.final_dict = {}

    def log_params(self, inputs_dict):
        self.param_dict = inputs_dict

    def _log(self, d, data):
        for k, v in data.items():
            d.setdefault(k, []).append(v)

    def log_train(self, data):
        self._log(self.train_dict, data)

    def log_eval(self, data):
        self._log(self.eval_dict, data)

    def log_final(self, data):
        self.final_dict.update(data)

    def dump(self):
        return {"param": self.param_dict, "train": self.train_dict, "eval": self.eval_dict, "final": self.final_dict}

    def save(self, path, name):
        os.makedirs(path, exist_ok=True)
        arrays = {}

        def conv(x, key):
            if isinstance(x, np.ndarray):
                arrays[key] = x
                return {"__npz__": key}
            if isinstance(x, dict):
                return {k: conv(v, f"{key}.{k}") for k, v in x.items()}
            if isinstance(x, (list, tuple)):
                return [conv(v, f"{key}.{i}") for i, v in enumerate(x)]
            if isinstance(x, (np.floating, np.integer)):
                return x.item()
            return x

        meta = conv(self.dump(), "log")
        with open(os.path.join(path, name + ".json"), "w") as fh:
            json.dump(meta, fh, default=str)
        if arrays:
            np.savez(os.path.join(path, name + ".npz"), **arrays)
        return os.path.join(path, name)
