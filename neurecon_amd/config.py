"""Attribute-access config dicts (the reference uses addict via utils/io_util.py:194-223)."""
import yaml


class Cfg(dict):
    """dict with attribute access; missing keys raise (like io_util.ForceKeyErrorDict)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def setdefault(self, k, default=None):
        if k not in self:
            self[k] = as_cfg(default)
        return self[k]


def as_cfg(d):
    if isinstance(d, Cfg):
        return d
    if isinstance(d, dict):
        c = Cfg()
        for k, v in d.items():
            dict.__setitem__(c, k, as_cfg(v))
        return c
    if isinstance(d, list):
        return [as_cfg(v) for v in d]
    return d


def load_yaml(path):
    with open(path) as f:
        return as_cfg(yaml.safe_load(f))
