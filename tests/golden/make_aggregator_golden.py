"""Generates tests/golden/aggregator_golden.json (+ aggregator_unit_test.npz).

The aggregation fixtures pin the learner-side batch aggregation byte for byte:
for each case, a seeded experience list in the reference senders' format
(oracle.aggregator_ref.make_*_exp_list; numpy RandomState streams are frozen
across numpy versions) goes through the oracle's loop-for-loop restatement of
surreal/learner/aggregator.py (MultistepAggregatorWithInfo :151-262,
SSARAggregator :52-103), and every output array is recorded as dtype, shape
and the SHA-256 of its bytes.  The reference --unit-test case (batch 2,
main/ppo_configs.py:225-227) is also stored in full (npz, no pickles).

Nothing here imports or runs the reference (denied: SURVEY.md §8(c)).
Run:  python tests/golden/make_aggregator_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import aggregator_ref as AR  # noqa: E402

PPO_CASES = [
    # name, B, T, D, A, rnn_hidden, pixel, seed
    ('unit_test_lstm', 2, 25, 17, 6, 100, None, 0),      # --unit-test: batch 2, default LSTM config
    ('c2_mlp', 64, 50, 17, 6, None, None, 1),            # BASELINE configs[1]
    ('c3_slice', 16, 25, 42, 8, 100, None, 2),           # C3 dims, 16 segments
    ('pixel_lstm', 3, 4, 5, 2, 8, (3, 12, 12), 3),       # low-dim + camera0 uint8
]
SSAR_CASES = [('c4_ssar', 64, 17, 6, 4)]


def digest(a):
    a = np.ascontiguousarray(a)
    return {'dtype': a.dtype.str, 'shape': list(a.shape),
            'sha256': hashlib.sha256(a.tobytes()).hexdigest()}


def flatten(out, prefix=''):
    """nested aggregate output -> {path: ndarray} (lists indexed, None kept as None)."""
    flat = {}
    if isinstance(out, dict):
        for k, v in out.items():
            flat.update(flatten(v, f'{prefix}{k}/'))
    elif isinstance(out, list):
        for i, v in enumerate(out):
            flat.update(flatten(v, f'{prefix}{i}/'))
    else:
        flat[prefix.rstrip('/')] = out
    return flat


def ppo_obs_spec(D, pixel):
    spec = {'low_dim': {'flat_inputs': (D,)}}
    if pixel is not None:
        spec['pixel'] = {'camera0': tuple(pixel)}
    return spec


def main():
    gold = {'ppo': {}, 'ssar': {}}
    for name, B, T, D, A, Hd, pixel, seed in PPO_CASES:
        arr = AR.ppo_exp_arrays(B, T, D, A, seed, rnn_hidden=Hd, pixel=pixel)
        out = AR.MultistepAggregatorWithInfoRef(ppo_obs_spec(D, pixel)).aggregate(
            AR.make_ppo_exp_list(arr))
        flat = flatten(out)
        gold['ppo'][name] = {'B': B, 'T': T, 'D': D, 'A': A, 'rnn_hidden': Hd,
                             'pixel': list(pixel) if pixel else None, 'seed': seed,
                             'outputs': {k: (None if v is None else digest(v))
                                         for k, v in flat.items()}}
        if name == 'unit_test_lstm':
            np.savez_compressed(os.path.join(HERE, 'aggregator_unit_test.npz'),
                                **{k.replace('/', '.'): v for k, v in flat.items() if v is not None})
    for name, B, D, A, seed in SSAR_CASES:
        arr = AR.ssar_exp_arrays(B, D, A, seed)
        out = AR.SSARAggregatorRef().aggregate(AR.make_ssar_exp_list(arr))
        gold['ssar'][name] = {'B': B, 'D': D, 'A': A, 'seed': seed,
                              'outputs': {k: digest(v) for k, v in flatten(out).items()}}
    with open(os.path.join(HERE, 'aggregator_golden.json'), 'w') as f:
        json.dump(gold, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
