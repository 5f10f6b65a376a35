"""Hand-derived rule -> node fixtures (test data, not code under test).

The reference has no tests for its rule -> node resolution, so
these cases were worked out by hand from the reference's code, not by running
the oracle or the engine:

* JobRule.included (job.go:274-288): a node is included when it is one of the
  rule's NodeIDs or a member (Group.Included, group.go:111-119) of one of its
  GroupIDs that exists; a missing group is skipped.
* Job.Cmds (job.go:591-614): nothing for a paused job; the ExcludeNodeIDs loop
  `continue`s only itself, so excludes change nothing; every included rule
  becomes cmds[Job.ID + Rule.ID] -- a later included rule with the same key
  replaces the earlier one (the map is per job: equal strings of two jobs do
  not collide).  Mode NONE.
* The engine's two further modes (cronsun_gpu.h cg_expand_per_node): RULE
  applies each rule's own ExcludeNodeIDs; CUMULATIVE applies the excludes of
  the rule and every earlier rule of its job -- web/job.go:222-257's
  GetJobNodes, per rule.  The Cmds key map applies on top in every mode.

Rules are numbered in job order then rule order (the engine's interned order).
EXPECTED[mode][node] = the rule indices scheduled on that node, ascending.
"""

CASES = [
    {
        "name": "groups_excludes_pause_keys",
        "groups": {"g1": ["n1", "n2"], "g2": ["n2", "n3"]},  # "gx" is referenced but missing
        "jobs": [
            {"id": "J1", "pause": False, "rules": [
                {"id": "a", "gids": ["g1"], "nids": ["n4"], "ex": ["n2"]},   # r0: g1 + n4 = n1 n2 n4
                {"id": "b", "gids": ["g2", "gx"], "nids": [], "ex": ["n3"]},  # r1: g2 = n2 n3 (gx skipped)
                {"id": "c", "gids": [], "nids": ["n3", "n5"], "ex": ["n1"]},  # r2: n3 n5
            ]},
            {"id": "J2", "pause": True, "rules": [
                {"id": "a", "gids": [], "nids": ["n1"], "ex": []},            # r3: paused job -> nowhere
            ]},
            {"id": "J3", "pause": False, "rules": [
                {"id": "x", "gids": [], "nids": ["n1", "n2"], "ex": []},      # r4: n1 n2
                {"id": "x", "gids": ["g2"], "nids": [], "ex": []},            # r5: n2 n3, same key J3x
                {"id": "y", "gids": [], "nids": [], "ex": []},                # r6: no nodes
            ]},
        ],
        "nodes": ["n1", "n2", "n3", "n4", "n5"],
        "expected": {
            # NONE: r0 {n1,n2,n4}, r1 {n2,n3}, r2 {n3,n5}, r4 {n1,n2}, r5 {n2,n3};
            # key J3x on n2: r5 (later) replaces r4
            "none": {"n1": [0, 4], "n2": [0, 1, 5], "n3": [1, 2, 5], "n4": [0], "n5": [2]},
            # RULE: r0 - n2 = {n1,n4}; r1 - n3 = {n2}; r2 - n1 = {n3,n5}
            "rule": {"n1": [0, 4], "n2": [1, 5], "n3": [2, 5], "n4": [0], "n5": [2]},
            # CUMULATIVE: r0 - {n2} = {n1,n4}; r1 - {n2,n3} = {}; r2 - {n2,n3,n1} = {n5}
            "cumulative": {"n1": [0, 4], "n2": [5], "n3": [5], "n4": [0], "n5": [2]},
        },
    },
    {
        "name": "blank_and_colliding_rule_ids",
        "groups": {"g": ["n1", "n3"]},
        "jobs": [
            {"id": "j", "pause": False, "rules": [
                {"id": "", "gids": [], "nids": ["n1", "n2"], "ex": []},     # r0: key "j"
                {"id": " ", "gids": [], "nids": ["n1"], "ex": []},          # r1: key "j " (never trimmed on this path)
                {"id": "", "gids": [], "nids": ["n2", "n3"], "ex": []},     # r2: key "j" again
                {"id": "1x", "gids": ["g"], "nids": [], "ex": []},          # r3: key "j1x"
            ]},
            {"id": "j1", "pause": False, "rules": [
                {"id": "x", "gids": [], "nids": ["n1"], "ex": []},          # r4: key "j1x" (job j1's own map)
                {"id": "x", "gids": ["g"], "nids": [], "ex": ["n1"]},       # r5: key "j1x"
            ]},
        ],
        "nodes": ["n1", "n2", "n3"],
        "expected": {
            # NONE: key "j" on n2: r2 replaces r0; key "j1x" of j1 on n1: r5
            # (excludes change nothing) replaces r4; j's "j1x" (r3) is kept apart
            "none": {"n1": [0, 1, 3, 5], "n2": [2], "n3": [2, 3, 5]},
            # RULE / CUMULATIVE: r5 excludes n1, so r4 keeps n1
            "rule": {"n1": [0, 1, 3, 4], "n2": [2], "n3": [2, 3, 5]},
            "cumulative": {"n1": [0, 1, 3, 4], "n2": [2], "n3": [2, 3, 5]},
        },
    },
]
