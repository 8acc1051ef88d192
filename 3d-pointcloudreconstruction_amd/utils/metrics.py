"""Evaluation metrics on the HIP path (counterpart of the reference's utils/metrics.py).

Surface kept from utils/metrics.py:10-109, so testnet.py-style callers work unchanged:

  * ``Metrics.ITEMS``: one descriptor per metric with the keys ``name``, ``enabled``,
    ``eval_func``, ``eval_object``, ``is_greater_better`` and ``init_value``. Callers
    may switch a metric off through ``enabled``.
  * ``Metrics.get(pred, gt)`` returns the enabled metrics' values as a list, in
    table order (EMD first, then CD; testnet.py:69 calls it this way).
  * ``Metrics.items()`` and ``Metrics.names()``.
  * ``Metrics._get_emd_distance``: 100 * mean over clouds of mean(sqrt(dist)) from
    the auction with eps 0.005 and 50 iterations (utils/metrics.py:49-53).
  * ``Metrics._get_chamfer_distance``: 100 * (mean(dist1) + mean(dist2))
    (utils/metrics.py:56-60).
  * ``Metrics(metric_name, values)``, where ``values`` is a list, or a dict keyed
    by metric name (unknown names are skipped with a warning). Also
    ``state_dict()``, ``repr()`` and ``better_than(other)``.

The reference builds its two modules with ``.cuda()`` when the class is defined
(:16, :24). The modules here hold no parameters or state, so no device is touched
at import time. All compute goes through libpcm_hip.so.
"""
import logging
import os
import sys

import torch

_METRIC_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "metric")
for _sub in ("emd", "chamfer3D"):
    _path = os.path.join(_METRIC_DIR, _sub)
    if _path not in sys.path:
        sys.path.append(_path)
from dist_chamfer_3D import chamfer_3DDist  # noqa: E402
import emd_module  # noqa: E402

# the evaluation call setting of utils/metrics.py:51 (the training loss uses 0.05 / 3000)
EVAL_EMD_EPS = 0.005
EVAL_EMD_ITERS = 50
_SCALE = 100.0

_log = logging.getLogger(__name__)


def _descriptor(name, method, module):
    # every metric here is a distance: lower is better, and 32767 is the
    # "not measured yet" placeholder of the reference table
    return dict(name=name, enabled=True, eval_func=method, eval_object=module,
                is_greater_better=False, init_value=32767)


class Metrics(object):
    ITEMS = [
        _descriptor('EMD_distance', '_get_emd_distance', emd_module.emdModule()),
        _descriptor('ChamferDistance', '_get_chamfer_distance', chamfer_3DDist()),
    ]

    # ---- class-level evaluation -------------------------------------------------
    @classmethod
    def items(cls):
        return list(filter(lambda d: d['enabled'], cls.ITEMS))

    @classmethod
    def names(cls):
        return [d['name'] for d in cls.items()]

    @classmethod
    def get(cls, pred, gt):
        return [getattr(cls, d['eval_func'])(pred, gt) for d in cls.items()]

    @classmethod
    def _module(cls, method):
        for d in cls.ITEMS:
            if d['eval_func'] == method:
                return d['eval_object']
        raise KeyError(method)

    @classmethod
    def _get_emd_distance(cls, pred, gt):
        dist, _ = cls._module('_get_emd_distance')(pred, gt, eps=EVAL_EMD_EPS, iters=EVAL_EMD_ITERS)
        per_cloud = dist.sqrt().mean(dim=1)
        return float(per_cloud.mean()) * _SCALE

    @classmethod
    def _get_chamfer_distance(cls, pred, gt):
        d1, d2, _, _ = cls._module('_get_chamfer_distance')(pred, gt)
        return float(d1.mean() + d2.mean()) * _SCALE

    # ---- a recorded set of metric values ---------------------------------------
    def __init__(self, metric_name, values):
        self.metric_name = metric_name
        self._items = Metrics.items()
        slot = {d['name']: i for i, d in enumerate(self._items)}
        if isinstance(values, list):
            self._values = values
        elif isinstance(values, dict):
            self._values = [d['init_value'] for d in self._items]
            for key, val in values.items():
                if key in slot:
                    self._values[slot[key]] = val
                else:
                    _log.warning('metric %r is not enabled; value dropped', key)
        else:
            raise Exception('Unsupported value type: %s' % type(values))

    def state_dict(self):
        return dict(zip((d['name'] for d in self._items), self._values))

    def __repr__(self):
        return repr(self.state_dict())

    def better_than(self, other):
        if other is None:
            return True
        pos = next((i for i, d in enumerate(self._items) if d['name'] == self.metric_name), None)
        if pos is None:
            raise Exception('Invalid metric name to compare.')
        mine, theirs = self._values[pos], other._values[pos]
        if self._items[pos]['is_greater_better']:
            return mine > theirs
        return mine < theirs
