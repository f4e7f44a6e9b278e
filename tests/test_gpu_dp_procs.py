"""The real data-parallel PPOLearner.learn() (dp=TorchDistAllReduce) in two
processes that share cuda:0 and exchange over torch.distributed (gloo here:
RCCL refuses two ranks on one GPU; on a multi-GPU node the same code runs over
'nccl' = RCCL/xGMI, as bench.py does).  Every rank must end with bit-identical
parameters, equal to the CPU oracle's learn() on the concatenated global batch
(tolerances as in test_gpu_ppo.py).  rnn='pixel' adds the camera + CNN stem
(SURVEY C5 structure, FC 32 wide) with one policy and one value epoch: over
more epochs the CNN's ReLU masks (pre-activations within fp32 noise of 0) and
Adam's sign-normalised first steps let any two fp32 implementations drift
apart by ~lr per affected entry (tools/dbg_px.py measures it)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B_LOC, T, D, A = 24, 10, 17, 6
CAM = (3, 84, 84)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(mode, rnn):
    from tests.helpers import ppo_config
    if rnn:
        return ppo_config(B=B_LOC, T=T, mode=mode, use_z_filter=True, hidden=(32, 48), lam=1.0,
                          rnn=True, rnn_hidden=40, horizon=3, cnn_feat=32,
                          epochs=(1, 1) if rnn == 'pixel' else (10, 10))
    return ppo_config(B=B_LOC, T=T, mode=mode, use_z_filter=True)


def _worker(rank, world, port, mode, outdir, rnn):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from surreal_amd import synthetic
    from surreal_amd.learner import PPOLearner, TorchDistAllReduce
    from surreal_amd.config import pixel_env_config
    from tests.helpers import env_config
    lc = _cfg(mode, rnn)
    ec = pixel_env_config(D, A, CAM) if rnn == 'pixel' else env_config(D, A)
    learner = PPOLearner(lc, ec, seed=21, device='cuda:0', dp=TorchDistAllReduce())
    init = {'actor': learner.model.actor.flat.cpu(), 'critic': learner.model.critic.flat.cpu()}
    if rnn:
        init['lstm'] = learner.model.rnn_stem.flat.cpu()
    if rnn == 'pixel':
        init['cnn'] = learner.model.cnn_stem.flat.cpu()
    res = []
    for it in range(2):
        full = synthetic.ppo_batch(B_LOC * world, T, D, A, seed=500 + it,
                                   rnn_hidden=40 if rnn else None,
                                   pixel=CAM if rnn == 'pixel' else None)
        dev = synthetic.to_device(full, 'cuda:0')
        lo, hi = rank * B_LOC, (rank + 1) * B_LOC

        def cut(x):
            if x is None:
                return None
            if isinstance(x, dict):
                return {k: cut(v) for k, v in x.items()}
            if isinstance(x, list):
                return [cut(v) for v in x]
            return x[lo:hi].contiguous()
        learner.learn(cut(dev))
        st = learner.last_stats()
        r = {'actor': learner.model.actor.flat.cpu(), 'critic': learner.model.critic.flat.cpu(),
             'zsum': learner.model.z_filter.running_sum.cpu(), 'stats': st}
        if rnn:
            r['lstm'] = learner.model.rnn_stem.flat.cpu()
        if rnn == 'pixel':
            r['cnn'] = learner.model.cnn_stem.flat.cpu()
        res.append(r)
    torch.save({'init': init, 'res': res}, os.path.join(outdir, f'rank{rank}.pt'))
    dist.destroy_process_group()


@pytest.mark.parametrize('mode,rnn', [('adapt', False), ('clip', False), ('adapt', True),
                                      ('clip', True), ('adapt', 'pixel')])
def test_two_process_dp_learn_matches_oracle(mode, rnn):
    from oracle import ppo_ref as R
    from surreal_amd import synthetic
    from tests.helpers import (load_lstm_flat, load_seq_flat, lstm_flat, max_rel_err, oracle_batch,
                               seq_flat)
    from tests.test_gpu_ppo import _compare_params
    world = 2
    with tempfile.TemporaryDirectory() as outdir:
        mp.spawn(_worker, args=(world, _free_port(), mode, outdir, rnn), nprocs=world, join=True)
        out = [torch.load(os.path.join(outdir, f'rank{r}.pt'), weights_only=True) for r in range(world)]
    lc = _cfg(mode, rnn)
    lc.replay.batch_size = B_LOC * world
    ref = R.PPOLearnerRef(lc, D, A, pixel=CAM if rnn == 'pixel' else None)
    ref.model.actor.load_flat(out[0]['init']['actor'])
    ref.model.critic.load_flat(out[0]['init']['critic'])
    ref.ref_target_model.actor.load_flat(out[0]['init']['actor'])
    ref.ref_target_model.critic.load_flat(out[0]['init']['critic'])
    if rnn:
        load_lstm_flat(ref.model.rnn_stem, out[0]['init']['lstm'])
        load_lstm_flat(ref.ref_target_model.rnn_stem, out[0]['init']['lstm'])
    if rnn == 'pixel':
        load_seq_flat(ref.model.cnn_stem, out[0]['init']['cnn'])
        load_seq_flat(ref.ref_target_model.cnn_stem, out[0]['init']['cnn'])
    report = {}
    for it in range(2):
        rstats = ref.learn(oracle_batch(synthetic.ppo_batch(B_LOC * world, T, D, A, seed=500 + it,
                                                            rnn_hidden=40 if rnn else None,
                                                            pixel=CAM if rnn == 'pixel' else None)))
        r0, r1 = out[0]['res'][it], out[1]['res'][it]
        assert torch.equal(r0['actor'], r1['actor']) and torch.equal(r0['critic'], r1['critic'])
        assert torch.equal(r0['zsum'], r1['zsum'])
        if rnn == 'pixel':
            assert torch.equal(r0['lstm'], r1['lstm']) and torch.equal(r0['cnn'], r1['cnn'])
            if it > 0:        # ranks agree; oracle distance drifts as described above
                continue
        assert r0['stats']['epochs_run'] == rstats['epochs_run']
        bad = [(k, r0['stats'][k], rstats[k]) for k in
               ('_surr_loss', '_pol_kl', '_entropy', '_val_loss', 'grad_norm_actor',
                'grad_norm_critic')
               if abs(r0['stats'][k] - rstats[k]) > 1e-4 * abs(rstats[k]) + 1e-6]
        print('stats mismatches', it, bad)
        _compare_params(f'actor{it}', r0['actor'], ref.model.actor.flat(), 3e-4,
                        rstats['epochs_run'], report)
        ev = lc.algo.consts.epoch_baseline
        _compare_params(f'critic{it}', r0['critic'], ref.model.critic.flat(), 3e-4, ev, report)
        if rnn:
            assert torch.equal(r0['lstm'], r1['lstm'])
            _compare_params(f'lstm{it}', r0['lstm'], lstm_flat(ref.model.rnn_stem), 3e-4,
                            rstats['epochs_run'] + ev, report)
        if rnn == 'pixel':
            _compare_params(f'cnn{it}', r0['cnn'], seq_flat(ref.model.cnn_stem), 3e-4,
                            rstats['epochs_run'] + ev, report, max_frac=5e-3)
        assert max_rel_err(r0['zsum'], ref.model.z_filter.running_sum) < 1e-5
        assert not bad, (it, bad)
    print('two-process dp report:', report)
