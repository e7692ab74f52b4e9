"""CPU tier: the FedAvg collective protocol (federated_multi_modal_amd/federated.py) and the federated
round loop (trainers.MaPLeFederated.train) across world_size 2, 3 and 8 gloo ranks, one client per rank,
checked against the reference's safe_average_weights / check_weights_valid semantics
(trainers/maple_fed.py:228-325, restated in oracle/maple_oracle.py and pinned to the reference by
tests/golden/fedavg.npz).

The device kernels are replaced by host restatements here (no GPU in this tier); the GPU tier
(tests/test_kernels_gpu.py) checks the kernels themselves against the same restatements."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import maple_oracle as O


class HostKernels:
    @staticmethod
    def nonfinite_flag(x, flag):
        if not torch.isfinite(x.float()).all():
            flag.fill_(1)

    @staticmethod
    def fedavg_pack(p16, p32, invalid, bucket):
        n16, n32 = p16.numel(), p32.numel()
        bad = bool(invalid.item())
        bucket[:n16] = 0.0 if bad else p16.float()
        bucket[n16:n16 + n32] = 0.0 if bad else p32
        bucket[n16 + n32] = 0.0 if bad else 1.0

    @staticmethod
    def fedavg_reduce_ordered(gathered, nclients, out):
        g = gathered.view(nclients, -1)[:, :out.numel()]
        acc = g[0].clone()
        for c in range(1, nclients):
            acc += g[c]
        out.copy_(acc)

    @staticmethod
    def fedavg_unpack(bucket, p16, p32, g16, g32):
        n16, n32 = p16.numel(), p32.numel()
        n_valid = float(bucket[n16 + n32])
        if n_valid == 0:
            p16.copy_(g16)
            p32.copy_(g32)
            return
        v = (bucket[: n16 + n32] / n_valid).half()
        p16.copy_(v[:n16])
        p32.copy_(v[n16:].float())
        g16.copy_(p16)
        g32.copy_(p32)


class FakeEngine:
    """flat16/flat32 trainables of one client; fp32 values spread over several binades so the fp32
    summation order of three clients shows in the fp16-rounded mean (~60 of the 1M elements differ
    between client order and a rotated order)."""

    def __init__(self, rank, n16=37, n32=(1 << 20) + 3, bad=False):
        g = torch.Generator().manual_seed(100 + rank)
        self.device = torch.device("cpu")
        self.n16, self.n32 = n16, n32
        self.flat16 = torch.randn(n16, generator=g).half()
        self.flat32 = torch.randn(n32, generator=g) * torch.exp2(torch.randint(-6, 6, (n32,), generator=g).float())
        if bad:
            self.flat32[3] = float("nan")
        self.reloaded = 0
        self.momentum_resets = 0

    def after_weights_loaded(self):
        self.reloaded += 1

    def reset_momentum(self):
        self.momentum_resets += 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker(rank, world, port, bad_ranks, mode, out):
    _init(rank, world, port)
    from federated_multi_modal_amd.federated import FedAvgBucket
    e = FakeEngine(rank, bad=rank in bad_ranks)
    g16, g32 = e.flat16.clone(), e.flat32.clone()
    e.flat16.copy_(FakeEngine(0).flat16)  # the previous global weights (identical on every rank)
    e.flat32.copy_(FakeEngine(0).flat32)
    fed = FedAvgBucket(e, kernels=HostKernels, mode=mode)
    e.flat16.copy_(g16)  # ... then this client's local training result
    e.flat32.copy_(g32)
    n_valid = fed.run()
    out[rank] = (n_valid, e.flat16.clone(), e.flat32.clone(), e.reloaded)
    dist.destroy_process_group()


def _spawn(fn, world, *args):  # noqa: D103
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(fn, args=(world, port) + args + (out,), nprocs=world, join=True)
    return dict(out)


@pytest.mark.parametrize("world,bad,mode", [(2, (), "ordered"), (3, (), "ordered"), (3, (1,), "ordered"),
                                            (2, (0, 1), "ordered"), (3, (), "allreduce"), (2, (1,), "allreduce"),
                                            # the federated configs' world size (C4 / C5: 8 clients on 8 ranks)
                                            (8, (), "ordered"), (8, (5,), "ordered")])
def test_fedavg_exchange_matches_reference(world, bad, mode):
    res = _spawn(_worker, world, tuple(bad), mode)
    clients = [FakeEngine(r, bad=r in bad) for r in range(world)]
    valid = [c for c in clients if O.check_weights_valid({"a": c.flat16, "b": c.flat32})]
    for r in range(world):
        n_valid, p16, p32, reloaded = res[r]
        assert n_valid == len(valid)
        assert reloaded == 1
        if not valid:  # all clients failed: round skipped, every client back to the previous global
            assert torch.equal(p16, FakeEngine(0).flat16) and torch.equal(p32, FakeEngine(0).flat32)
            continue
        ref = O.safe_average_weights([{"a": c.flat16, "b": c.flat32} for c in valid])
        if mode == "ordered":  # client-order fp32 sums: bit-exact at any world size
            assert torch.equal(p16, ref["a"])
            assert torch.equal(p32, ref["b"].float())
        else:  # collective order: within one fp16 ulp
            ulp = torch.exp2(torch.floor(torch.log2(ref["b"].float().abs().clamp_min(2.0 ** -14))) - 10)
            assert ((p32 - ref["b"].float()).abs() <= ulp).all()
            assert torch.equal(p16, ref["a"]) or world > 2
    # every rank holds the same global weights (broadcast-free exchange)
    assert all(torch.equal(res[0][1], res[r][1]) and torch.equal(res[0][2], res[r][2]) for r in range(world))


def _group_worker(rank, world, port, per_rank, bad, mode, out):
    """Several clients per rank (clients rank*C .. rank*C + C - 1) through one FedAvgExchange."""
    _init(rank, world, port)
    from federated_multi_modal_amd.federated import FedAvgBucket, FedAvgExchange
    ids = list(range(rank * per_rank, (rank + 1) * per_rank))
    engines = [FakeEngine(c, bad=c in bad) for c in ids]
    feds = []
    for e in engines:
        loc16, loc32 = e.flat16.clone(), e.flat32.clone()
        e.flat16.copy_(FakeEngine(0).flat16)
        e.flat32.copy_(FakeEngine(0).flat32)
        feds.append(FedAvgBucket(e, kernels=HostKernels, mode=mode))
        e.flat16.copy_(loc16)
        e.flat32.copy_(loc32)
    x = FedAvgExchange(feds, mode=mode)
    for f in feds:
        f.pack()
    x.start()
    x.finish([])
    for f in feds:
        f.unpack()
    out[rank] = (feds[0].n_valid(), [(e.flat16.clone(), e.flat32.clone()) for e in engines])
    dist.destroy_process_group()


@pytest.mark.parametrize("world,per_rank,bad,mode", [(2, 2, (), "ordered"), (3, 2, (4,), "ordered"),
                                                     (2, 3, (), "allreduce")])
def test_fedavg_several_clients_per_rank(world, per_rank, bad, mode):
    """FED.NUM_CLIENTS a multiple of WORLD_SIZE: every client of every rank ends with
    safe_average_weights over all valid clients -- bit for bit in the ordered mode (the all_to_all delivers
    [source rank][local client] = the reference's client order)."""
    res = _spawn(_group_worker, world, per_rank, tuple(bad), mode)
    clients = [FakeEngine(c, bad=c in bad) for c in range(world * per_rank)]
    valid = [c for c in clients if O.check_weights_valid({"a": c.flat16, "b": c.flat32})]
    ref = O.safe_average_weights([{"a": c.flat16, "b": c.flat32} for c in valid])
    for r in range(world):
        n_valid, weights = res[r]
        assert n_valid == len(valid)
        for p16, p32 in weights:
            if mode == "ordered":
                assert torch.equal(p16, ref["a"]) and torch.equal(p32, ref["b"].float())
            else:  # another fp32 summation order: one fp16 ulp, plus fp32 cancellation of the largest inputs
                ulp = torch.exp2(torch.floor(torch.log2(ref["b"].float().abs().clamp_min(2.0 ** -14))) - 10)
                big = torch.stack([c.flat32.abs() for c in valid]).max(0).values
                assert ((p32 - ref["b"].float()).abs() <= ulp + 1e-6 * big).all()


# ----------------------------------------------------------------------------- the round loop itself

class _Optim:
    def __init__(self):
        self.lr = 1e-3
        self.sched = None

    def rebuild(self, epoch):
        pass


class FakeClient:
    """Stands in for MaPLe (one client per rank) in MaPLeFederated.train(): run_epoch "trains" by a
    deterministic per-(client, round, epoch) update, fails with the reference's RuntimeError when told,
    calls before_test exactly where MaPLe.run_epoch does, and logs the order of events."""

    def __init__(self, rank, fail_rounds=(), late_fail_rounds=(), abort_round=None):
        self.client_id = rank
        self.engine = FakeEngine(0)  # every client starts from the same global weights
        self.optim = _Optim()
        self.sched = None
        self.fail_rounds = set(fail_rounds)
        self.late_fail_rounds = set(late_fail_rounds)  # test() of the last epoch raises (after FedAvg started)
        self.abort_round = abort_round                 # a ValueError (not caught by the reference) that round
        self.events = []
        self.model = self
        # MaPLe.timing's counters (trainers.py): 3 "steps" per completed local epoch
        self.timing = {"train_s": 0.0, "test_s": 0.0, "fedavg_launch_s": 0.0, "steps": 0, "epochs": 0}

    def state_dict(self):
        return {"flat16": self.engine.flat16, "flat32": self.engine.flat32}

    @staticmethod
    def local_update(rank, round_idx, ep, e):
        g = torch.Generator().manual_seed(1000 * rank + 100 * round_idx + ep)
        e.flat16 += (1e-2 * torch.randn(e.n16, generator=g)).half()
        e.flat32 += 1e-3 * torch.randn(e.n32, generator=g) * e.flat32.abs()

    def run_epoch(self, ep, before_test=None):
        round_idx = ep // 2
        if round_idx in self.fail_rounds and ep % 2 == 1:
            self.events.append(("fail", ep))
            raise RuntimeError("NaN/Inf in total loss")
        if round_idx == self.abort_round:
            self.events.append(("abort", ep))
            raise ValueError("NaN/Inf values in input image")
        self.local_update(self.client_id, round_idx, ep, self.engine)
        self.timing["steps"] += 3
        self.timing["epochs"] += 1
        if before_test is not None:
            self.events.append(("fedavg_start", ep))
            before_test()
        self.events.append(("test", ep))
        if before_test is not None and round_idx in self.late_fail_rounds:
            raise RuntimeError("kernel failure in test()")
        return {"avg_loss": 1.0}

    def test(self, evaluate_train=False):
        self.events.append(("global_test", None))
        return {"accuracy": 50.0}


def _train_worker(rank, world, port, per_rank, fail, late, abort, out):
    _init(rank, world, port)
    from federated_multi_modal_amd.config import extend_cfg, get_cfg_default
    from federated_multi_modal_amd.federated import FedAvgBucket, FedAvgExchange
    from federated_multi_modal_amd.trainers import MaPLeFederated
    cfg = get_cfg_default()
    extend_cfg(cfg)
    cfg.OUTPUT_DIR = f"/tmp/mapfed_fedtest_{port}"
    tr = MaPLeFederated.__new__(MaPLeFederated)   # the round loop without building GPU engines
    tr.cfg, tr.num_clients, tr.num_rounds, tr.local_epochs = cfg, world * per_rank, 2, 2
    tr.nan_stats = {"total_updates": 0, "failed_clients": [], "skipped_rounds": 0}
    tr.distributed, tr.rank = True, rank
    ids = list(range(rank * per_rank, (rank + 1) * per_rank))
    tr.clients = [FakeClient(c, fail_rounds=fail.get(c, ()), late_fail_rounds=late.get(c, ()),
                             abort_round=abort.get(c)) for c in ids]
    tr.fed = [FedAvgBucket(c.engine, kernels=HostKernels, mode="ordered") for c in tr.clients]
    tr.exchange = FedAvgExchange(tr.fed, mode="ordered")
    tr.save_model = lambda *a, **k: None
    err = None
    try:
        tr.train()
    except Exception as exc:  # noqa: BLE001 - the abort cases end here on every rank
        err = f"{type(exc).__name__}: {exc}"
    out[rank] = ([(c.engine.flat16.clone(), c.engine.flat32.clone()) for c in tr.clients],
                 [list(c.events) for c in tr.clients], dict(tr.nan_stats),
                 [c.engine.momentum_resets for c in tr.clients], err, list(getattr(tr, "round_times", [])))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,per_rank,fail,late", [
    (2, 1, {}, {}), (3, 1, {1: (0,)}, {}), (2, 1, {0: (1,), 1: (1,)}, {}),
    (2, 2, {1: (0,)}, {}),                 # 4 clients on 2 ranks, trained two after another per rank
    (2, 1, {}, {1: (1,)}), (2, 2, {}, {0: (0,), 3: (1,)}),  # a client's last test() fails after its bucket went out
    (8, 1, {3: (0,)}, {6: (1,)}),          # world 8 (C4 / C5: one client per GPU of the node), one bad rank per round
])
def test_round_loop_distributed(world, per_rank, fail, late):
    """MaPLeFederated.train() on gloo ranks: 2 rounds x 2 local epochs; each client's bucket is packed inside
    its last local epoch, after the SGD steps and before that epoch's test() (the rank's last client starts
    the exchange there: the overlap), and the global weights after every round equal safe_average_weights
    over the clients that did not fail, bit for bit -- also for a client whose last test() raises after
    its bucket went out; an all-failed round keeps the previous global weights
    (trainers/maple_fed.py:247-303)."""
    res = _spawn(_train_worker, world, per_rank, fail, late, {})
    n = world * per_rank
    # expected: replay the rounds on the host with the reference's aggregation
    g16, g32 = FakeEngine(0).flat16.clone(), FakeEngine(0).flat32.clone()
    for r in range(2):
        locals_ = []
        for c in range(n):
            e = FakeEngine(0)
            e.flat16.copy_(g16)
            e.flat32.copy_(g32)
            failed = r in fail.get(c, ())
            for ep in (2 * r, 2 * r + 1):
                if failed and ep % 2 == 1:
                    break
                FakeClient.local_update(c, r, ep, e)
            if not failed and r not in late.get(c, ()):
                locals_.append({"a": e.flat16, "b": e.flat32})
        if locals_:
            avg = O.safe_average_weights(locals_)
            g16, g32 = avg["a"], avg["b"].float()
    for rank in range(world):
        weights, events, stats, resets, err, rounds = res[rank]
        assert err is None, err
        # MaPLeFederated.round_times: one record per round, its phases inside the round's wall time
        assert [r["round"] for r in rounds] == [1, 2]
        for ri, r in enumerate(rounds):
            phases = ("local_train_s", "local_test_s", "fedavg_launch_s", "fedavg_exposed_s", "global_state_s",
                      "global_test_s", "other_s")
            # other_s is the remainder, so the sum holds by construction: every phase must also be >= 0 (no phase
            # double-counted), and the step / epoch counts must be the rank's completed local epochs
            assert all(r[k] >= 0.0 for k in phases), r
            assert abs(sum(r[k] for k in phases) - r["wall_s"]) < 1e-6 and r["clients"] == per_rank
            epochs = sum(2 - (1 if ri in fail.get(c, ()) else 0) for c in range(rank * per_rank, (rank + 1) * per_rank))
            assert r["epochs"] == epochs and r["steps"] == 3 * epochs, (r, epochs)
        for j, (p16, p32) in enumerate(weights):
            c = rank * per_rank + j
            assert torch.equal(p16, g16) and torch.equal(p32, g32), c
            assert resets[j] == 2  # broadcast_weights drops the SGD momentum every round
            ev = events[j]
            for r in range(2):
                if r in fail.get(c, ()):
                    assert ("fail", 2 * r + 1) in ev
                    continue
                i = ev.index(("fedavg_start", 2 * r + 1))
                assert ev[i + 1] == ("test", 2 * r + 1)      # the exchange overlaps the last local test
                assert ("fedavg_start", 2 * r) not in ev       # packed once per round, in the last epoch
        local_failed = sum(len(fail.get(c, ())) + len(late.get(c, ())) for c in range(rank * per_rank,
                                                                                     (rank + 1) * per_rank))
        assert len(stats["failed_clients"]) == local_failed
    skipped = sum(1 for r in range(2) if all(r in fail.get(c, ()) or r in late.get(c, ()) for c in range(n)))
    assert res[0][2]["skipped_rounds"] == skipped and res[0][2]["total_updates"] == 2 - skipped


def test_round_loop_abort_stops_every_rank():
    """A non-finite input raises ValueError on one rank (trainers/maple.py:526-535; the reference does not
    catch it and its process dies): every rank leaves train() at that round's exchange -- the failing rank
    with its ValueError, its peers with FederatedAbort -- instead of waiting in the next round's collectives."""
    res = _spawn(_train_worker, 3, 1, {}, {}, {1: 1})
    assert res[1][4].startswith("ValueError")
    assert res[0][4].startswith("FederatedAbort") and res[2][4].startswith("FederatedAbort")
    for rank in range(3):
        assert res[rank][2]["total_updates"] == 1   # round 0 completed everywhere


def test_exchange_launch_failure_is_not_retried_as_a_client_failure():
    """A FedAvg collective that fails to launch inside the last client's epoch hook propagates out of train()
    (its cause re-raised) instead of being taken for a client failure: the round loop does not pack the bucket
    again as 'failed' and does not launch the exchange a second time on this rank alone (which would leave the
    peers in mismatched collectives).  One process, the exchange replaced by a stub that fails on start()."""
    from federated_multi_modal_amd.config import extend_cfg, get_cfg_default
    from federated_multi_modal_amd.federated import FedAvgBucket
    from federated_multi_modal_amd.trainers import MaPLeFederated

    class FailingExchange:
        def __init__(self):
            self.starts = 0

        def start(self):
            self.starts += 1
            raise RuntimeError("collective launch failed")

        def finish(self, *a, **k):
            raise AssertionError("finish() must not run after a failed launch")

    cfg = get_cfg_default()
    extend_cfg(cfg)
    tr = MaPLeFederated.__new__(MaPLeFederated)
    tr.cfg, tr.num_clients, tr.num_rounds, tr.local_epochs = cfg, 1, 2, 2
    tr.nan_stats = {"total_updates": 0, "failed_clients": [], "skipped_rounds": 0}
    tr.distributed, tr.rank = False, 0
    tr.clients = [FakeClient(0)]
    tr.fed = [FedAvgBucket(tr.clients[0].engine, kernels=HostKernels, mode="ordered")]
    packs = []
    orig_pack = tr.fed[0].pack
    tr.fed[0].pack = lambda failed=False: (packs.append(failed), orig_pack(failed=failed))
    tr.exchange = FailingExchange()
    tr.save_model = lambda *a, **k: None
    with pytest.raises(RuntimeError, match="collective launch failed"):
        tr.train()
    assert tr.exchange.starts == 1 and packs == [False]
    assert tr.nan_stats["failed_clients"] == []
