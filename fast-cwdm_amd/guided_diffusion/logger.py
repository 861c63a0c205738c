"""Key/value logger with the API TrainLoop uses (guided_diffusion/logger.py:
logkv, logkv_mean, dumpkvs, log/warn, configure).  stdout / log.txt /
progress.csv outputs; wandb and TensorBoard are out of scope."""
import csv
import os
import sys
from collections import defaultdict

DEBUG, INFO, WARN, ERROR, DISABLED = 10, 20, 30, 40, 50


class Logger:
    def __init__(self, dir=None, format_strs=("stdout",)):
        self.dir = dir
        self.level = INFO
        self.name2val = defaultdict(float)
        self.name2cnt = defaultdict(int)
        self.formats = list(format_strs)
        self._csv_keys = None
        if dir:
            os.makedirs(dir, exist_ok=True)

    def logkv(self, key, val):
        self.name2val[key] = val

    def logkv_mean(self, key, val):
        oldval, cnt = self.name2val[key], self.name2cnt[key]
        self.name2val[key] = oldval * cnt / (cnt + 1) + val / (cnt + 1)
        self.name2cnt[key] = cnt + 1

    def dumpkvs(self):
        d = dict(self.name2val)
        if self.level < DISABLED and d:
            if "stdout" in self.formats:
                width = max(len(k) for k in d)
                lines = [f"| {k:<{width}} | {v:<12.6g} |" if isinstance(v, float) else f"| {k:<{width}} | {v!s:<12} |"
                         for k, v in sorted(d.items())]
                sys.stdout.write("\n".join(lines) + "\n")
                sys.stdout.flush()
            if "csv" in self.formats and self.dir:
                path = os.path.join(self.dir, "progress.csv")
                keys = sorted(d)
                new = self._csv_keys != keys
                with open(path, "a", newline="") as f:
                    w = csv.writer(f)
                    if new:
                        w.writerow(keys)
                        self._csv_keys = keys
                    w.writerow([d[k] for k in keys])
        self.name2val.clear()
        self.name2cnt.clear()
        return d

    def log(self, *args, level=INFO):
        if self.level <= level:
            msg = " ".join(map(str, args))
            sys.stdout.write(msg + "\n")
            if self.dir and "log" in self.formats:
                with open(os.path.join(self.dir, "log.txt"), "a") as f:
                    f.write(msg + "\n")


_current = Logger()


def configure(dir=None, format_strs=None, comm=None, log_suffix=""):
    global _current
    _current = Logger(dir, tuple(format_strs) if format_strs else ("stdout", "log", "csv"))
    return _current


def get_current():
    return _current


def logkv(key, val):
    _current.logkv(key, val)


def logkv_mean(key, val):
    _current.logkv_mean(key, val)


def logkvs(d):
    for k, v in d.items():
        logkv(k, v)


def dumpkvs():
    return _current.dumpkvs()


def getkvs():
    return _current.name2val


def log(*args, level=INFO):
    _current.log(*args, level=level)


def debug(*args):
    log(*args, level=DEBUG)


def info(*args):
    log(*args, level=INFO)


def warn(*args):
    log(*args, level=WARN)


def error(*args):
    log(*args, level=ERROR)


def set_level(level):
    _current.level = level


def get_dir():
    return _current.dir
