"""Evaluation metrics -- working counterpart of the reference's utils/metrics.py.

Same ``Metrics`` class surface (utils/metrics.py:10-109): ITEMS, get, items,
names, _get_emd_distance (EMD x100 with eps=0.005, iters=50) and
_get_chamfer_distance (CD x100), state_dict, better_than.  The metric modules
are constructed at class-definition time as in the reference (:16, :24);
they hold no parameters, so this needs no device.
"""
import logging
import os
import sys

import torch

_METRIC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "metric")
for _p in (os.path.join(_METRIC, "emd"), os.path.join(_METRIC, "chamfer3D")):
    if _p not in sys.path:
        sys.path.append(_p)
from dist_chamfer_3D import chamfer_3DDist  # noqa: E402
import emd_module as emd_func  # noqa: E402


class Metrics(object):
    ITEMS = [{
        'name': 'EMD_distance',
        'enabled': True,
        'eval_func': '_get_emd_distance',
        'eval_object': emd_func.emdModule(),
        'is_greater_better': False,
        'init_value': 32767
    }, {
        'name': 'ChamferDistance',
        'enabled': True,
        'eval_func': '_get_chamfer_distance',
        'eval_object': chamfer_3DDist(),
        'is_greater_better': False,
        'init_value': 32767
    }]

    @classmethod
    def get(cls, pred, gt):
        _items = cls.items()
        _values = [0] * len(_items)
        for i, item in enumerate(_items):
            _values[i] = getattr(cls, item['eval_func'])(pred, gt)
        return _values

    @classmethod
    def items(cls):
        return [i for i in cls.ITEMS if i['enabled']]

    @classmethod
    def names(cls):
        return [i['name'] for i in cls.items()]

    @classmethod
    def _get_emd_distance(cls, pred, gt):
        emd_distance = cls.ITEMS[0]['eval_object']
        emd_1, _ = emd_distance(pred, gt, eps=0.005, iters=50)
        emd_loss = torch.sqrt(emd_1).mean(1).mean()
        return emd_loss.item() * 100

    @classmethod
    def _get_chamfer_distance(cls, pred, gt):
        chamfer_distance = cls.ITEMS[1]['eval_object']
        dist1, dist2, idx1, idx2 = chamfer_distance(pred, gt)
        chamfer_loss = torch.mean(dist1) + torch.mean(dist2)
        return chamfer_loss.item() * 100

    def __init__(self, metric_name, values):
        self._items = Metrics.items()
        self._values = [item['init_value'] for item in self._items]
        self.metric_name = metric_name

        if type(values).__name__ == 'list':
            self._values = values
        elif type(values).__name__ == 'dict':
            metric_indexes = {}
            for idx, item in enumerate(self._items):
                metric_indexes[item['name']] = idx
            for k, v in values.items():
                if k not in metric_indexes:
                    logging.warning('Ignore Metric[Name=%s] due to disability.' % k)
                    continue
                self._values[metric_indexes[k]] = v
        else:
            raise Exception('Unsupported value type: %s' % type(values))

    def state_dict(self):
        return {self._items[i]['name']: self._values[i] for i in range(len(self._items))}

    def __repr__(self):
        return str(self.state_dict())

    def better_than(self, other):
        if other is None:
            return True
        _index = -1
        for i, _item in enumerate(self._items):
            if _item['name'] == self.metric_name:
                _index = i
                break
        if _index == -1:
            raise Exception('Invalid metric name to compare.')
        _metric = self._items[_index]
        _value = self._values[_index]
        other_value = other._values[_index]
        return _value > other_value if _metric['is_greater_better'] else _value < other_value
