"""Seeded synthetic rule sets for the BASELINE.json configs.

spec_mix(n, seed)          config 2 mix of cron.Parse spec strings
rules_for_nodes(...)       config 3 jobs x groups x nodes (integer-interned)
"""
import numpy as np

from .engine import RulesIn

T0_2026 = 1767571200  # 2026-01-05T00:00:00Z
MONTHS = ["Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"]
DOWS = ["Sun", "Mon", "Tue", "Wed", "Thu", "Fri", "Sat"]

# (name, fraction) -- config 2 ("1M rules mixed specs"), SURVEY.md §8d-2
MIX_CONFIG2 = [
    ("minute", 0.25),      # minute-level steps/lists
    ("daily", 0.20),       # hourly/daily fixed times with dow ranges
    ("domdow", 0.10),      # dom and dow both restricted (OR semantics)
    ("month", 0.10),       # month-restricted / descriptors
    ("every", 0.15),       # @every, D log-uniform in [30 s, 6 h]
    ("second", 0.10),      # second granularity
    ("never", 0.05),       # never fires (Feb 30, Apr 31)
    ("mixed", 0.05),       # ranges and steps mixed
]
# config 3/4: same families, second granularity reduced (bounds fan-out volume)
MIX_LIGHT = [("minute", 0.25), ("daily", 0.25), ("domdow", 0.10), ("month", 0.10),
             ("every", 0.15), ("second", 0.01), ("never", 0.05), ("mixed", 0.09)]


def _minute(rng):
    k = rng.integers(0, 4)
    if k == 0:
        return f"0 */{rng.choice([1, 2, 5, 10, 15, 20, 30])} * * * *"
    if k == 1:
        a = sorted(rng.choice(60, size=rng.integers(2, 5), replace=False))
        h0 = int(rng.integers(0, 12))
        return f"0 {','.join(map(str, a))} {h0}-{h0 + int(rng.integers(4, 12))} * * *"
    if k == 2:
        return f"{rng.integers(0, 60)} {rng.integers(0, 15)}/{rng.choice([5, 10, 15])} * * * *"
    return f"0 */{rng.choice([2, 3, 5, 7, 13])} {rng.integers(0, 8)}-23 * * {rng.integers(0, 3)}-{rng.integers(4, 7)}"


def _daily(rng):
    k = rng.integers(0, 3)
    m, h = int(rng.integers(0, 60)), int(rng.integers(0, 24))
    if k == 0:
        return f"0 {m} {h} * * {rng.integers(0, 3)}-{rng.integers(3, 7)}"
    if k == 1:
        return f"0 {m} * * * *"
    return f"{rng.integers(0, 60)} {m} {h},{(h + 12) % 24} * * *"


def _domdow(rng):
    d = sorted(rng.choice(np.arange(1, 29), size=2, replace=False))
    return f"0 {rng.integers(0, 60)} {rng.integers(0, 24)} {d[0]},{d[1]} * {DOWS[rng.integers(0, 7)]}"


def _month(rng):
    k = rng.integers(0, 7)
    if k == 0:
        return "@daily"
    if k == 1:
        return "@weekly"
    if k == 2:
        return "@monthly"
    if k == 3:
        return "@hourly"
    if k == 4:
        a, b = sorted(rng.choice(12, size=2, replace=False))
        return f"0 0 0 1 {MONTHS[a]},{MONTHS[b]} ?"
    if k == 5:
        return f"0 30 {rng.integers(0, 24)} * {MONTHS[rng.integers(0, 6)]}-{MONTHS[rng.integers(6, 12)]} *"
    return "@yearly"


def _every(rng):
    d = int(np.exp(rng.uniform(np.log(30), np.log(6 * 3600))))
    h, rem = divmod(d, 3600)
    m, s = divmod(rem, 60)
    out = ""
    if h:
        out += f"{h}h"
    if m:
        out += f"{m}m"
    if s or not out:
        out += f"{s}s"
    return "@every " + out


def _second(rng):
    k = rng.integers(0, 3)
    if k == 0:
        return f"*/{rng.choice([5, 10, 15, 20, 30])} * * * * *"
    if k == 1:
        return f"{rng.integers(0, 30)}/{rng.integers(20, 45)} * * * * *"
    return f"*/{rng.choice([10, 30])} {rng.integers(0, 30)}-59 {rng.integers(0, 12)}-23 * * *"


def _never(rng):
    return ["0 0 0 30 Feb ?", "0 0 0 31 Apr ?", "0 0 0 31 Jun,Sep,Nov ?"][rng.integers(0, 3)]


def _mixed(rng):
    return (f"{rng.integers(0, 30)}/{rng.integers(10, 40)} {rng.integers(0, 30)}-{rng.integers(30, 60)}/"
            f"{rng.integers(1, 20)} {rng.integers(0, 12)}/{rng.integers(1, 6)} */{rng.integers(1, 4)} * *")


GEN = {"minute": _minute, "daily": _daily, "domdow": _domdow, "month": _month,
       "every": _every, "second": _second, "never": _never, "mixed": _mixed}


def spec_mix(n, seed=0x5EED, mix=MIX_CONFIG2, every_second_frac=0.001):
    """n spec strings of the given mix (deterministic for a seed)."""
    rng = np.random.default_rng(seed)
    names = [m[0] for m in mix]
    p = np.array([m[1] for m in mix], dtype=np.float64)
    kinds = rng.choice(len(names), size=n, p=p / p.sum())
    out = []
    star = rng.random(n) < every_second_frac
    for i in range(n):
        out.append("* * * * * *" if star[i] else GEN[names[kinds[i]]](rng))
    return out


def rules_for_nodes(n_rules, n_nodes=10000, n_groups=500, seed=0x5EED + 3,
                    group_size=(4, 256), max_gids=3, max_nids=4, max_ex=2, pause_frac=0.01,
                    missing_group_frac=0.01):
    """Config 3: one rule per job; groups of log-uniform size; 0-3 GroupIDs,
    0-4 NodeIDs, 0-2 ExcludeNodeIDs per rule."""
    rng = np.random.default_rng(seed)
    sizes = np.exp(rng.uniform(np.log(group_size[0]), np.log(group_size[1]), n_groups)).astype(np.int64)
    group_off = np.zeros(n_groups + 1, dtype=np.int64)
    group_off[1:] = np.cumsum(sizes)
    group_nodes = np.concatenate([rng.choice(n_nodes, size=s, replace=False) for s in sizes]).astype(np.int32)
    group_exists = (rng.random(n_groups) >= missing_group_frac).astype(np.uint8)

    def lists(maxk, lim):
        k = rng.integers(0, maxk + 1, n_rules)
        off = np.zeros(n_rules + 1, dtype=np.int64)
        off[1:] = np.cumsum(k)
        vals = rng.integers(0, lim, int(off[-1])).astype(np.int32)
        return off, vals

    gid_off, gids = lists(max_gids, n_groups)
    nid_off, nids = lists(max_nids, n_nodes)
    ex_off, ex = lists(max_ex, n_nodes)
    return RulesIn(n_nodes, n_groups, n_rules, n_rules,
                   group_off=group_off, group_nodes=group_nodes, group_exists=group_exists,
                   rule_job=np.arange(n_rules, dtype=np.int32), nid_off=nid_off, nids=nids,
                   gid_off=gid_off, gids=gids, ex_off=ex_off, ex=ex,
                   job_pause=(rng.random(n_rules) < pause_frac).astype(np.uint8))


def multi_rule_jobs(n_jobs, rules_per_job=(1, 4), n_nodes=64, n_groups=12, seed=7, key_choices=0):
    """Small jobsets with several rules per job (exclude-mode semantics tests).
    key_choices > 0: each rule's Rule.ID is one of that many values (rule_key),
    so rules of a job repeat Cmd keys (Job.Cmds keeps the last, job.go:604-609)."""
    rng = np.random.default_rng(seed)
    per = rng.integers(rules_per_job[0], rules_per_job[1] + 1, n_jobs)
    rule_job = np.repeat(np.arange(n_jobs, dtype=np.int32), per)
    R = int(per.sum())
    base = rules_for_nodes(R, n_nodes=n_nodes, n_groups=n_groups, seed=seed + 1,
                           group_size=(2, max(3, n_nodes // 3)), max_gids=2, max_nids=3, max_ex=3,
                           pause_frac=0.0)
    base.rule_job = rule_job
    base.n_jobs = n_jobs
    base.job_pause = (rng.random(n_jobs) < 0.1).astype(np.uint8)
    if key_choices:
        base.rule_key = rng.integers(0, key_choices, R).astype(np.int32)
    return base
