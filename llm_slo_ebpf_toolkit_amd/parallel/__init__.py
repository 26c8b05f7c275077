"""Multi-GPU scaling for the window engine: one process per MI355X, RCCL over xGMI.

* ``dist``     -- process-group bring-up from torchrun env (nccl == RCCL on GPUs, gloo for
                  CPU tests), 127.0.0.1 rendezvous defaults.
* ``shard``    -- P1 event-stream data parallelism: records are owned by the rank that owns
                  their node (REF runs one agent per node).
* ``exchange`` -- exact cross-shard joins: trace-tagged events are all-gathered so tier-1
                  (trace id) matches that cross nodes are found (REF's per-node agents miss
                  them), and P2 time halos carry the last ``outer`` ns of the previous window
                  into the next so streaming windows join like one unbounded batch. Imported
                  records sit after the node-local ones and are excluded from the window's
                  counters (``counts[3] = n_local`` in the decode kernels), so the packed
                  all-reduce still counts every event exactly once.
* P3 overlap lives in pipeline/window.py (copy / compute / RCCL streams).
"""
