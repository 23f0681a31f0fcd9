"""`torch.utils.tensorboard.SummaryWriter` stand-in.

torch.utils.tensorboard needs the `tensorboard` package, which is not in this image;
experiments/ppo_gridnet.py:20 imports SummaryWriter from it and calls
add_text / add_scalar / close (ppo_gridnet.py:349-352, 487-490, 600-615).
gym_microrts.run_driver installs this module as `torch.utils.tensorboard` only when
the real import fails.  Scalars and text go to `<log_dir>/events.jsonl`, one JSON
object per call ({"tag", "value", "step", "wall_time"}).
"""
import json
import os
import time

__microrts_compat__ = True


class SummaryWriter:
    def __init__(self, log_dir=None, comment="", **kwargs):
        if log_dir is None:
            log_dir = os.path.join("runs", time.strftime("%b%d_%H-%M-%S") + comment)
        self.log_dir = log_dir
        os.makedirs(log_dir, exist_ok=True)
        self._f = open(os.path.join(log_dir, "events.jsonl"), "a")

    def _write(self, kind, tag, value, step, walltime):
        if self._f is None:
            return
        self._f.write(json.dumps({"kind": kind, "tag": tag, "value": value, "step": step,
                                  "wall_time": walltime if walltime is not None else time.time()}) + "\n")

    def add_scalar(self, tag, scalar_value, global_step=None, walltime=None, **kwargs):
        v = scalar_value.item() if hasattr(scalar_value, "item") else float(scalar_value)
        self._write("scalar", tag, v, None if global_step is None else int(global_step), walltime)

    def add_scalars(self, main_tag, tag_scalar_dict, global_step=None, walltime=None):
        for k, v in tag_scalar_dict.items():
            self.add_scalar(f"{main_tag}/{k}", v, global_step, walltime)

    def add_text(self, tag, text_string, global_step=None, walltime=None):
        self._write("text", tag, str(text_string), global_step, walltime)

    def add_histogram(self, tag, values, global_step=None, **kwargs):
        import numpy as np

        a = values.detach().cpu().numpy() if hasattr(values, "detach") else np.asarray(values)
        self._write("histogram", tag, {"min": float(a.min()), "max": float(a.max()), "mean": float(a.mean())},
                    global_step, None)

    def flush(self):
        if self._f is not None:
            self._f.flush()

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
