"""Row compaction bookkeeping (batching.plan_compaction) on CPU: the moves a BatchSynthesizer
issues through mx_llm_move_row when streams end, and the host rows they leave behind."""
from project_morpheus_amd.batching import _Row, plan_compaction


def _rows(spec):
    """spec: one char per row: '.' free, 'L' live, 'P' parked, 'S' stopped."""
    rows = []
    for i, c in enumerate(spec):
        r = _Row(i)
        if c != ".":
            r.req = object()
            r.slot = 100 + i   # KV slot: fixed for the stream's life
            r.parked = c == "P"
            r.stopped = c == "S"
        rows.append(r)
    return rows


def _state(rows):
    assert all(r.idx == i for i, r in enumerate(rows))
    return "".join("." if r.req is None else ("P" if r.parked else "S" if r.stopped else "L")
                   for r in rows)


def test_highest_live_row_moves_into_lowest_free_row():
    rows = _rows(".LL.L")
    reqs = [r.req for r in rows]
    slot_of = {id(r.req): r.slot for r in rows if r.req is not None}
    moves = plan_compaction(rows)
    assert moves == [(0, 4)]
    assert _state(rows) == "LLL.."
    assert rows[0].req is reqs[4] and rows[0].slot == slot_of[id(reqs[4])]
    assert plan_compaction(rows) == []          # idempotent


def test_several_moves_fill_every_hole_in_order():
    rows = _rows("..L.LL")
    assert plan_compaction(rows) == [(0, 5), (1, 4)]
    assert _state(rows) == "LLL..."


def test_parked_and_stopped_rows_stay_put_and_never_move():
    rows = _rows("P.SL")
    assert plan_compaction(rows) == [(1, 3)]
    assert _state(rows) == "PLS."
    rows = _rows(".PS")        # nothing live: no step runs, nothing to move
    assert plan_compaction(rows) == []
    assert _state(rows) == ".PS"


def test_no_move_when_live_rows_are_a_prefix():
    for spec in ("LLL", "LL..", "L.P", ""):
        rows = _rows(spec)
        assert plan_compaction(rows) == []
        assert _state(rows) == spec


def test_row_class_after_compaction_is_the_live_count():
    rows = _rows("L" * 32)
    for i in range(0, 32, 2):      # every other stream ends
        rows[i].req = None
    plan_compaction(rows)
    live = [r for r in rows if r.req is not None and not r.parked and not r.stopped]
    assert max(r.idx for r in live) + 1 == 16
