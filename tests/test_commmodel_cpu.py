"""The step model of the gradient synchronisation modes (parallel/commmodel.py,
docs/COMM_MODEL.md): wire bytes per mode, the forward-time x gather, the per-weight best plan."""
from tutorial_torch_distributed_data_parallel_amd.parallel import commmodel as cm


def _wire(W, mode):
    layers = cm.toy_mlp_layers(128)
    r = cm.simulate(layers, {"fc1": mode, "fc2": mode}, W, 128, cm.Hardware())
    return sum(j["wire_MB"] for j in r["jobs"]), r


def test_wire_bytes_per_mode():
    # all-reduce of the 218 MB gradient moves 2 (W-1)/W of it per rank
    ar, _ = _wire(8, "allreduce")
    assert abs(ar - 2 * 7 / 8 * 4 * (9216 * 4096 + 4096 * 4096) / 1e6) < 1.0
    rep, _ = _wire(8, "factored-replicated")
    shd, _ = _wire(8, "factored-sharded")
    # factors only (W*B rows of g and x) < factors + parameter all-gather < gradient all-reduce
    assert rep < shd < ar
    assert abs(rep - 7 / 8 * 4 * 1024 * (9216 + 4096 + 4096 + 4096) / 1e6) < 1.0


def test_forward_x_gather_shortens_the_tail():
    layers = cm.toy_mlp_layers(128)
    modes = {"fc1": "factored-sharded", "fc2": "factored-sharded"}
    hw = cm.Hardware()
    early = cm.simulate(layers, modes, 8, 128, hw, prefetch_x=True)
    late = cm.simulate(layers, modes, 8, 128, hw, prefetch_x=False)
    assert early["exposed_us"] < late["exposed_us"]


def test_early_g_gather_precedes_the_parameter_all_gather():
    # fc1's g gathered from fc2's backward (after fc2's gated input-gradient GEMM) instead of
    # queueing behind fc2's parameter all-gather on the side stream
    layers = cm.toy_mlp_layers(128)
    hw = cm.Hardware()
    for W, mode in ((2, "factored-replicated"), (8, "factored-split"), (8, "factored-sharded")):
        modes = {"fc1": mode, "fc2": mode}
        on = cm.simulate(layers, modes, W, 128, hw, early_g=True)
        off = cm.simulate(layers, modes, W, 128, hw, early_g=False)
        assert on["step_us"] < off["step_us"], (W, mode)
        fc1 = {j["layer"]: j for j in on["jobs"]}["fc1"]
        fc1_off = {j["layer"]: j for j in off["jobs"]}["fc1"]
        assert fc1["start_us"] < fc1_off["start_us"]
    # bucket-mode neighbours have no factors to gather early: nothing changes
    modes = {"fc1": "allreduce", "fc2": "allreduce"}
    assert cm.simulate(layers, modes, 8, 128, hw, early_g=True)["step_us"] == \
        cm.simulate(layers, modes, 8, 128, hw, early_g=False)["step_us"]


def test_best_plan_beats_uniform_plans_and_follows_bandwidth():
    layers = cm.toy_mlp_layers(128)
    for W in (2, 4, 8):
        best = cm.best_plan(layers, W, 128, cm.Hardware())
        for mode in cm.MODES:
            r = cm.simulate(layers, {"fc1": mode, "fc2": mode}, W, 128, cm.Hardware())
            assert best["step_us"] <= r["step_us"] + 1e-6
    # a slow link makes the parameter all-gather expensive: replication wins
    slow = cm.Hardware(busbw_GBps={"all_gather": 20.0, "all_reduce": 20.0, "reduce_scatter": 20.0})
    b = cm.best_plan(layers, 8, 128, slow)
    for j in b["jobs"]:  # replicated, or split with most rows replicated
        assert j["mode"] in ("factored-replicated", "factored-split"), b
        assert j["rep_fraction"] > 0.75, b


def test_split_mode_hides_the_parameter_all_gather_at_w8():
    """The headline at W=8 (assumed xGMI: 7 links x 51 GB/s): replicating part of the rows while
    the rest is all-gathered beats both pure modes (docs/COMM_MODEL.md)."""
    layers = cm.toy_mlp_layers(128)
    hw = cm.Hardware()
    r = {m: cm.simulate(layers, {"fc1": m, "fc2": m}, 8, 128, hw)["step_us"]
         for m in ("factored-sharded", "factored-replicated", "factored-split")}
    assert r["factored-split"] < 0.8 * min(r["factored-sharded"], r["factored-replicated"]), r


def test_one_rank_has_no_communication():
    layers = cm.toy_mlp_layers(128)
    r = cm.simulate(layers, {"fc1": "allreduce", "fc2": "allreduce"}, 1, 128, cm.Hardware())
    assert all(j["wire_MB"] == 0 for j in r["jobs"])


def test_table_rows():
    rows = cm.table((2, 8))
    assert len(rows) == 2 * (len(cm.MODES) + 1)
    assert all(r["step_us"] >= r["exposed_us"] >= 0 for r in rows)


def test_cnn_bucket_model_resnet50():
    """BASELINE config 5: ResNet-50's bucketed gradient sync hides behind its 22 ms backward
    except the last bucket (the stem / layer1 gradients arrive last); a smaller bucket cap
    shrinks that tail on xGMI (docs/COMM_MODEL.md)."""
    fwd, grads = cm.cnn_grads("resnet50")
    assert len(grads) == 161 and sum(g.numel for g in grads) == 23_528_522
    t = cm.CNN_DP1_MS["resnet50"]
    assert abs(sum(g.bwd_us for g in grads) - 1e3 * (2 * t["gemm"] / 3 + t["bn_bwd"])) < 1.0
    assert grads[0].name.startswith("fc.") and grads[-1].name in ("conv1.weight", "bn1.weight")
    hw = cm.Hardware()
    exp = {cap: cm.simulate_buckets(fwd, grads, 2, hw, cap_mb=cap)["exposed_us"]
           for cap in (4, 25, 64, 1024)}
    assert exp[4] <= exp[25] <= exp[64] <= exp[1024] and exp[1024] > 1000.0, exp
    r8 = cm.simulate_buckets(fwd, grads, 8, hw)  # the default plan: 1 MiB first, 25 MiB
    assert r8["exposed_us"] < 0.01 * r8["compute_us"], r8


def test_tensor_sharded_model_beats_factored_at_w8():
    """The tensor-sharded step (activations over xGMI) against the best factored plan at W = 8
    under the same assumed hardware: shorter predicted step, >= 70 % of dp1, and the chunked
    overlap hides part of its two big collectives."""
    hw = cm.Hardware()
    t1 = cm.simulate_tensor(8, hw=hw)
    t4 = cm.simulate_tensor(8, hw=hw, chunks=4)
    fac = cm.best_plan(cm.toy_mlp_layers(), 8, 128, hw)
    assert t1["step_us"] < fac["step_us"]
    assert t1["scaling_eff"] >= 0.70 and t4["exposed_us"] < t1["exposed_us"]
    # gathering the node's batch locally saves the 33 MB input all-gather
    assert cm.simulate_tensor(8, hw=hw, global_batch=False)["step_us"] > t1["step_us"] + 90
    assert cm.simulate_tensor(1)["exposed_us"] == 0.0


def test_factored_bound_is_below_every_simulated_plan():
    """factored_bound: no simulated DDP plan beats the schedule-independent bound, and at W = 8
    the bound itself stays under 70 % of the dp1 model step at the default link figure
    (docs/COMM_MODEL.md "What ANY DDP schedule can reach")."""
    from tutorial_torch_distributed_data_parallel_amd.parallel import commmodel as cm

    L = cm.toy_mlp_layers(128)
    hw = cm.Hardware()
    alone = sum(x.fwd_us + x.dgrad_us + x.wgrad_us for x in L)
    for W in (2, 4, 8):
        b = cm.factored_bound(L, W, 128, hw)
        assert b["step_us"] == max(b["compute_us"], b["wire_us"])
        for m1 in cm.MODES[2:]:
            for m2 in cm.MODES[2:]:
                r = cm.simulate(L, {"fc1": m1, "fc2": m2}, W, 128, hw)
                assert r["step_us"] >= b["step_us"] - 1.0, (W, m1, m2, r["step_us"], b)
    assert alone / cm.factored_bound(L, 8, 128, hw)["step_us"] < 0.70
