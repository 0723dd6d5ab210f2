"""Logger with the reference's layout (``sac_eo/common/logger.py:5-91``): dict-of-lists
``train`` data, ``param`` inputs and ``final`` weights / normaliser stats, saved as the
reference's pickle ``{'param', 'train', 'final'}`` with the train arrays of an existing file
in front (``dump_and_save``, ``:57-86``), so the reference's analysis tooling reads our logs.

``load_log`` reads such a file (ours, or one the reference wrote) with an allow-list
unpickler: only containers, scalars and NumPy array / dtype reconstruction are resolved;
any other global in the file is refused, so loading a log executes nothing from it."""
import os
import pickle

import numpy as np

# (module, name) globals a log may reference: NumPy's array / scalar reconstruction
# (numpy 1.x pickles name numpy.core, numpy 2.x numpy._core); protocol 5 pickles contiguous
# arrays through numeric._frombuffer, which only builds an array from bytes
_ALLOWED = {(m, n) for m in ("numpy.core.multiarray", "numpy._core.multiarray")
            for n in ("_reconstruct", "scalar")} | {("numpy", "ndarray"), ("numpy", "dtype")} | \
           {(m, "_frombuffer") for m in ("numpy.core.numeric", "numpy._core.numeric")}
# written with protocol 4 so the file does not depend on the interpreter's default protocol
PICKLE_PROTOCOL = 4


class _LogUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"log file references {module}.{name}: refused (not a sac_eo log)")


def load_log(filename):
    """A sac_eo log file: the dict of one run's checkpoint, or the list of runs that
    ``train.py`` aggregates (reference ``sac_eo/train.py:159-186``)."""
    with open(filename, "rb") as fh:
        return _LogUnpickler(fh).load()


class Logger:
    """Class for logging data throughout training (reference ``logger.py:5-91``)."""

    def __init__(self):
        self.param_dict = dict()
        self.train_dict = dict()
        self.final_dict = dict()

    def log_train(self, kv):
        for k, v in kv.items():
            self.train_dict.setdefault(k, []).append(v)

    def log_train_ensemble(self, kv_list):
        ens = dict()
        for kv in kv_list:
            for k, v in kv.items():
                ens.setdefault(k, []).append(v)
        self.log_train({k: np.array(v) for k, v in ens.items()})

    def log_params(self, kv):
        for k, v in kv.items():
            self.param_dict[k] = v

    def log_final(self, kv):
        for k, v in kv.items():
            self.final_dict[k] = v

    def dump(self):
        return {"param": self.param_dict, "train": {k: np.array(v) for k, v in self.train_dict.items()},
                "final": self.final_dict}

    def dump_and_save(self, log_path, log_name):
        """Writes ``{'param', 'train', 'final'}``; train arrays already in the file come first.
        An existing file that cannot be read (or merged) is overwritten, as the reference's
        bare ``except: pass`` does (``logger.py:71-83``)."""
        out = self.dump()
        os.makedirs(log_path, exist_ok=True)
        filename = os.path.join(log_path, log_name)
        try:
            old = load_log(filename)
            merged = dict(out["train"])
            for k, v in old["train"].items():
                merged[k] = np.concatenate((v, out["train"][k]), axis=0) if k in out["train"] else v
            out["train"] = merged
        except (OSError, EOFError, pickle.UnpicklingError, KeyError, TypeError, ValueError, AttributeError):
            pass
        with open(filename, "wb") as fh:
            pickle.dump(out, fh, protocol=PICKLE_PROTOCOL)
        return filename

    def reset(self):
        self.param_dict.clear()
        self.train_dict.clear()
        self.final_dict.clear()
