"""Property tests of the A2A task lifecycle store (facade/a2a.py): under random
state requests and cancels, only the transitions of ``isValidTransition``
(internal/facade/a2a/redis_task_store.go:379-395) happen, terminal tasks never
change, every accepted change reaches a subscriber once and in order, and the
bounded store evicts only terminal tasks."""
import asyncio

from hypothesis import given, settings
from hypothesis import strategies as st

from omnia_amd.facade.a2a import (TERMINAL, TRANSITIONS, InvalidTransition, MemoryTaskStore,
                                  TaskNotFound)

STATES = ["working", "completed", "failed", "canceled", "input-required", "auth-required",
          "rejected", "submitted"]


@given(st.lists(st.tuples(st.integers(0, 3), st.sampled_from(STATES + ["<cancel>"])),
                max_size=60),
       st.integers(2, 6))
@settings(max_examples=200, deadline=None)
def test_task_store_lifecycle(ops, max_tasks):
    async def run():
        store = MemoryTaskStore(max_tasks=max_tasks)
        tasks, subs, seen, state = {}, {}, {}, {}
        for i in range(4):
            tasks[i] = await store.create(f"t{i}", "ctx", {"role": "user", "parts": []})
            subs[i] = await store.subscribe(f"t{i}")
            seen[i] = []
            state[i] = "submitted"
        for i, want in ops:
            cur = state[i]
            try:
                if want == "<cancel>":
                    await store.cancel(f"t{i}")
                    new = "canceled"
                else:
                    await store.set_state(tasks[i], want)
                    new = want
            except InvalidTransition:
                assert (("canceled" if want == "<cancel>" else want)
                        not in TRANSITIONS.get(cur, ()))
                continue
            except TaskNotFound:  # a terminal task the bounded store evicted: stays gone
                assert cur in TERMINAL and await store.get(f"t{i}") is None
                continue
            assert cur not in TERMINAL
            assert new in TRANSITIONS[cur]
            seen[i].append(new)
            state[i] = new
        for i in range(4):
            got = []
            while True:
                ev = await subs[i].get(timeout=0.01)
                if ev is None:
                    break
                got.append(ev)
            assert got == seen[i]
            subs[i].close()
            t = await store.get(f"t{i}")
            if t is None:  # evicted: only ever a terminal task
                assert seen[i] and seen[i][-1] in TERMINAL
        live = [t for t in store.tasks.values() if t["status"]["state"] not in TERMINAL]
        assert len(store.tasks) <= max(max_tasks, len(live))

    asyncio.run(run())
