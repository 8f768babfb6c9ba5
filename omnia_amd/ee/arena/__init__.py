"""Arena: evaluation / load-test jobs (reference ``ee/cmd/arena-worker``,
``ee/pkg/arena``, ``ee/internal/controller`` arena reconcilers).

* :mod:`.queue`     -- work items on Redis Streams (consumer groups, reclaim) or in memory
* :mod:`.profile`   -- ramp-up / ramp-down load profile
* :mod:`.fleet`     -- WebSocket client against an agent facade, measures TTFT + turn latency
* :mod:`.worker`    -- virtual-user pool executing scenario x provider work items
* :mod:`.stats`     -- aggregation + threshold evaluation (latency/TTFT percentiles,
                       error/pass rate, cost, tokens/s)
* :mod:`.controller`-- ArenaJob reconciler (partition -> enqueue -> workers -> verdict)
"""
