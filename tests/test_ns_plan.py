"""Host logic of the NS trainer's lookahead pipeline (regnn_hip.ns.plan_run / warm_walk, no GPU):
every replay run_steps plans trains only slots the sampler has filled and refills only slots
already trained, and capture()'s warm walk launches every captured graph once."""
import itertools
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "re-gnn_amd"))
from regnn_hip.ns import group_sizes, plan_run, warm_walk  # noqa: E402


def test_group_sizes():
    assert group_sizes(8) == [8, 4, 2]
    assert group_sizes(4) == [4, 2]
    assert group_sizes(1) == []


def _simulate(ahead, plan, cur):
    """slot states: sampled (ready to train) or stale; a step at slot c trains c and samples
    c + ahead (mod 2 ahead). A group of m from c: all of c .. c+m-1 sampled before, all of
    c+ahead .. c+ahead+m-1 stale (trained) before."""
    n = 2 * ahead
    ready = {(cur + i) % n for i in range(ahead)}
    for m, start in plan:
        assert start == cur
        train = [(start + i) % n for i in range(m)]
        fill = [(start + ahead + i) % n for i in range(m)]
        assert all(s in ready for s in train)
        assert not set(fill) & ready and not set(fill) & set(train)
        ready -= set(train)
        ready |= set(fill)
        cur = (cur + m) % n
        assert ready == {(cur + i) % n for i in range(ahead)}
    return cur


@pytest.mark.parametrize("order", ["desc", "asc", "lead4", "lead2"])
@pytest.mark.parametrize("ahead", [2, 4, 8])
def test_plan_run_keeps_the_sampled_window(ahead, order):
    n = 2 * ahead
    for cur, k in itertools.product(range(n), range(1, 3 * n + 2)):
        plan = plan_run(cur, k, ahead, n, order=order)
        assert sum(m for m, _ in plan) == k
        assert all(m == 1 or m in group_sizes(ahead) for m, _ in plan)
        assert len(plan) <= k // ahead + len(group_sizes(ahead)) + 2
        end = _simulate(ahead, plan, cur)
        assert end == (cur + k) % n


def test_plan_run_without_a_group_falls_back_to_single_steps():
    plan = plan_run(3, 8, 8, 16, have=lambda m, c: c != 3, order="desc")
    assert plan[0] == (1, 3) and plan[1][1] == 4 and sum(m for m, _ in plan) == 8


def test_plan_orders():
    from regnn_hip.ns import plan_sizes
    assert plan_sizes(20, 32, "desc") == [16, 4]
    assert plan_sizes(20, 32, "asc") == [4, 16]
    assert plan_sizes(20, 32, "lead4") == [4, 16]
    assert plan_sizes(160, 32, "lead4") == [4, 32, 32, 32, 32, 16, 8, 4]
    assert plan_sizes(3, 32, "lead4") == [2, 1]


@pytest.mark.parametrize("ahead", [2, 4, 8])
def test_warm_walk_visits_every_graph(ahead):
    n = 2 * ahead
    walk = warm_walk(ahead, n)
    groups = {(m, c) for m, c in walk if m > 1}
    singles = {c for m, c in walk if m == 1}
    assert groups == {(m, c) for m in group_sizes(ahead) for c in range(n)}
    assert singles == set(range(n))
    _simulate(ahead, walk, 0)
