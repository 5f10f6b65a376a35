"""Generate tests/golden/kats.json: the reference's own known-answer tables
for the scheduling path, transcribed as data (inputs + expected outputs).

Sources (qlchan/cronsun, /root/reference):
  node/cron/spec_test.go:8-71     TestActivation   (29 rows)
  node/cron/spec_test.go:73-167   TestNext         (41 rows)
  node/cron/spec_test.go:169-182  TestErrors       (4 rows)
  node/cron/spec_test.go:206-231  TestNextWithTz   (4 rows)
  node/cron/constantdelay_test.go:8-54 TestConstantDelayNext (14 rows)
  node/cron/parser_test.go        TestRange (20) TestField (4) TestAll (5)
                                  TestBits (4) TestParse (8)
                                  TestStandardSpecSchedule (4)

Time strings are converted to unix seconds the way the tests' getTime /
getTimeTZ helpers do (spec_test.go:184-249): the "Mon Jan 2 15:04[:05] 2006"
layouts are UTC; the "2006-01-02T15:04:05-0700" layout is an instant that
getTime moves into America/New_York and getTimeTZ keeps in a fixed zone of the
parsed offset.  The empty string is Go's zero time (-62135596800).

Run:  python tests/golden/gen_kats.py   (writes kats.json next to this file)
"""
import datetime as dt
import json
import os

ZERO = -62135596800
STAR = 1 << 63


def parse_time(s):
    """-> (unix, nsec, offset_or_None)"""
    if s == "":
        return ZERO, 0, None
    for layout in ("%a %b %d %H:%M %Y", "%a %b %d %H:%M:%S %Y"):
        try:
            t = dt.datetime.strptime(s, layout).replace(tzinfo=dt.timezone.utc)
            return int(t.timestamp()), 0, None
        except ValueError:
            pass
    # fractional seconds after the seconds field (Go accepts them when parsing)
    if "." in s and not s[0].isdigit():
        head, rest = s.split(".", 1)
        frac, year = rest.split(" ", 1)
        t = dt.datetime.strptime(head + " " + year, "%a %b %d %H:%M:%S %Y")
        t = t.replace(tzinfo=dt.timezone.utc)
        nsec = int(frac.ljust(9, "0"))
        return int(t.timestamp()), nsec, None
    t = dt.datetime.strptime(s, "%Y-%m-%dT%H:%M:%S%z")
    return int(t.timestamp()), 0, int(t.utcoffset().total_seconds())


# ---- spec_test.go:13-55 TestActivation: (line, time, spec, expected) ----
ACTIVATION = [
    (14, "Mon Jul 9 15:00 2012", "0 0/15 * * *", True),
    (15, "Mon Jul 9 15:45 2012", "0 0/15 * * *", True),
    (16, "Mon Jul 9 15:40 2012", "0 0/15 * * *", False),
    (19, "Mon Jul 9 15:05 2012", "0 5/15 * * *", True),
    (20, "Mon Jul 9 15:20 2012", "0 5/15 * * *", True),
    (21, "Mon Jul 9 15:50 2012", "0 5/15 * * *", True),
    (24, "Sun Jul 15 15:00 2012", "0 0/15 * * Jul", True),
    (25, "Sun Jul 15 15:00 2012", "0 0/15 * * Jun", False),
    (28, "Sun Jul 15 08:30 2012", "0 30 08 ? Jul Sun", True),
    (29, "Sun Jul 15 08:30 2012", "0 30 08 15 Jul ?", True),
    (30, "Mon Jul 16 08:30 2012", "0 30 08 ? Jul Sun", False),
    (31, "Mon Jul 16 08:30 2012", "0 30 08 15 Jul ?", False),
    (34, "Mon Jul 9 15:00 2012", "@hourly", True),
    (35, "Mon Jul 9 15:04 2012", "@hourly", False),
    (36, "Mon Jul 9 15:00 2012", "@daily", False),
    (37, "Mon Jul 9 00:00 2012", "@daily", True),
    (38, "Mon Jul 9 00:00 2012", "@weekly", False),
    (39, "Sun Jul 8 00:00 2012", "@weekly", True),
    (40, "Sun Jul 8 01:00 2012", "@weekly", False),
    (41, "Sun Jul 8 00:00 2012", "@monthly", False),
    (42, "Sun Jul 1 00:00 2012", "@monthly", True),
    (46, "Sun Jul 15 00:00 2012", "0 * * 1,15 * Sun", True),
    (47, "Fri Jun 15 00:00 2012", "0 * * 1,15 * Sun", True),
    (48, "Wed Aug 1 00:00 2012", "0 * * 1,15 * Sun", True),
    (51, "Sun Jul 15 00:00 2012", "0 * * * * Mon", False),
    (52, "Sun Jul 15 00:00 2012", "0 * * */10 * Sun", False),
    (53, "Mon Jul 9 00:00 2012", "0 * * 1,15 * *", False),
    (54, "Sun Jul 15 00:00 2012", "0 * * 1,15 * *", True),
    (55, "Sun Jul 15 00:00 2012", "0 * * */2 * Sun", True),
]

# ---- spec_test.go:79-152 TestNext: (line, time, spec, expected) ----
NEXT = [
    (79, "Mon Jul 9 14:45 2012", "0 0/15 * * *", "Mon Jul 9 15:00 2012"),
    (80, "Mon Jul 9 14:59 2012", "0 0/15 * * *", "Mon Jul 9 15:00 2012"),
    (81, "Mon Jul 9 14:59:59 2012", "0 0/15 * * *", "Mon Jul 9 15:00 2012"),
    (84, "Mon Jul 9 15:45 2012", "0 20-35/15 * * *", "Mon Jul 9 16:20 2012"),
    (87, "Mon Jul 9 23:46 2012", "0 */15 * * *", "Tue Jul 10 00:00 2012"),
    (88, "Mon Jul 9 23:45 2012", "0 20-35/15 * * *", "Tue Jul 10 00:20 2012"),
    (89, "Mon Jul 9 23:35:51 2012", "15/35 20-35/15 * * *", "Tue Jul 10 00:20:15 2012"),
    (90, "Mon Jul 9 23:35:51 2012", "15/35 20-35/15 1/2 * *", "Tue Jul 10 01:20:15 2012"),
    (91, "Mon Jul 9 23:35:51 2012", "15/35 20-35/15 10-12 * *", "Tue Jul 10 10:20:15 2012"),
    (93, "Mon Jul 9 23:35:51 2012", "15/35 20-35/15 1/2 */2 * *", "Thu Jul 11 01:20:15 2012"),
    (94, "Mon Jul 9 23:35:51 2012", "15/35 20-35/15 * 9-20 * *", "Wed Jul 10 00:20:15 2012"),
    (95, "Mon Jul 9 23:35:51 2012", "15/35 20-35/15 * 9-20 Jul *", "Wed Jul 10 00:20:15 2012"),
    (98, "Mon Jul 9 23:35 2012", "0 0 0 9 Apr-Oct ?", "Thu Aug 9 00:00 2012"),
    (99, "Mon Jul 9 23:35 2012", "0 0 0 */5 Apr,Aug,Oct Mon", "Mon Aug 6 00:00 2012"),
    (100, "Mon Jul 9 23:35 2012", "0 0 0 */5 Oct Mon", "Mon Oct 1 00:00 2012"),
    (103, "Mon Jul 9 23:35 2012", "0 0 0 * Feb Mon", "Mon Feb 4 00:00 2013"),
    (104, "Mon Jul 9 23:35 2012", "0 0 0 * Feb Mon/2", "Fri Feb 1 00:00 2013"),
    (107, "Mon Dec 31 23:59:45 2012", "0 * * * * *", "Tue Jan 1 00:00:00 2013"),
    (110, "Mon Jul 9 23:35 2012", "0 0 0 29 Feb ?", "Mon Feb 29 00:00 2016"),
    (113, "2012-03-11T00:00:00-0500", "0 30 2 11 Mar ?", "2013-03-11T02:30:00-0400"),
    (116, "2012-03-11T00:00:00-0500", "0 0 * * * ?", "2012-03-11T01:00:00-0500"),
    (117, "2012-03-11T01:00:00-0500", "0 0 * * * ?", "2012-03-11T03:00:00-0400"),
    (118, "2012-03-11T03:00:00-0400", "0 0 * * * ?", "2012-03-11T04:00:00-0400"),
    (119, "2012-03-11T04:00:00-0400", "0 0 * * * ?", "2012-03-11T05:00:00-0400"),
    (122, "2012-03-11T00:00:00-0500", "0 0 1 * * ?", "2012-03-11T01:00:00-0500"),
    (123, "2012-03-11T01:00:00-0500", "0 0 1 * * ?", "2012-03-12T01:00:00-0400"),
    (126, "2012-03-11T00:00:00-0500", "0 0 2 * * ?", "2012-03-12T02:00:00-0400"),
    (129, "2012-11-04T00:00:00-0400", "0 30 2 04 Nov ?", "2012-11-04T02:30:00-0500"),
    (130, "2012-11-04T01:45:00-0400", "0 30 1 04 Nov ?", "2012-11-04T01:30:00-0500"),
    (133, "2012-11-04T00:00:00-0400", "0 0 * * * ?", "2012-11-04T01:00:00-0400"),
    (134, "2012-11-04T01:00:00-0400", "0 0 * * * ?", "2012-11-04T01:00:00-0500"),
    (135, "2012-11-04T01:00:00-0500", "0 0 * * * ?", "2012-11-04T02:00:00-0500"),
    (138, "2012-11-04T00:00:00-0400", "0 0 1 * * ?", "2012-11-04T01:00:00-0400"),
    (139, "2012-11-04T01:00:00-0400", "0 0 1 * * ?", "2012-11-04T01:00:00-0500"),
    (140, "2012-11-04T01:00:00-0500", "0 0 1 * * ?", "2012-11-05T01:00:00-0500"),
    (143, "2012-11-04T00:00:00-0400", "0 0 2 * * ?", "2012-11-04T02:00:00-0500"),
    (144, "2012-11-04T02:00:00-0500", "0 0 2 * * ?", "2012-11-05T02:00:00-0500"),
    (147, "2012-11-04T00:00:00-0400", "0 0 3 * * ?", "2012-11-04T03:00:00-0500"),
    (148, "2012-11-04T03:00:00-0500", "0 0 3 * * ?", "2012-11-05T03:00:00-0500"),
    (151, "Mon Jul 9 23:35 2012", "0 0 0 30 Feb ?", ""),
    (152, "Mon Jul 9 23:35 2012", "0 0 0 31 Apr ?", ""),
]

# ---- spec_test.go:171-174 TestErrors ----
ERRORS = [(171, "xyz"), (172, "60 0 * * *"), (173, "0 60 * * *"), (174, "0 0 * * XYZ")]

# ---- spec_test.go:212-217 TestNextWithTz ----
NEXT_TZ = [
    (212, "2016-01-03T13:09:03+0530", "0 14 14 * * *", "2016-01-03T14:14:00+0530"),
    (213, "2016-01-03T04:09:03+0530", "0 14 14 * * ?", "2016-01-03T14:14:00+0530"),
    (216, "2016-01-03T14:09:03+0530", "0 14 14 * * *", "2016-01-03T14:14:00+0530"),
    (217, "2016-01-03T14:00:00+0530", "0 14 14 * * ?", "2016-01-03T14:14:00+0530"),
]

NS = 1
US = 1000
MS = 1000 * US
S = 1000 * MS
M = 60 * S
H = 60 * M

# ---- constantdelay_test.go:15-44 TestConstantDelayNext: (line, time, delay_ns, expected) ----
CONST_DELAY = [
    (15, "Mon Jul 9 14:45 2012", 15 * M + 50 * NS, "Mon Jul 9 15:00 2012"),
    (16, "Mon Jul 9 14:59 2012", 15 * M, "Mon Jul 9 15:14 2012"),
    (17, "Mon Jul 9 14:59:59 2012", 15 * M, "Mon Jul 9 15:14:59 2012"),
    (20, "Mon Jul 9 15:45 2012", 35 * M, "Mon Jul 9 16:20 2012"),
    (23, "Mon Jul 9 23:46 2012", 14 * M, "Tue Jul 10 00:00 2012"),
    (24, "Mon Jul 9 23:45 2012", 35 * M, "Tue Jul 10 00:20 2012"),
    (25, "Mon Jul 9 23:35:51 2012", 44 * M + 24 * S, "Tue Jul 10 00:20:15 2012"),
    (26, "Mon Jul 9 23:35:51 2012", 25 * H + 44 * M + 24 * S, "Thu Jul 11 01:20:15 2012"),
    (29, "Mon Jul 9 23:35 2012", 91 * 24 * H + 25 * M, "Thu Oct 9 00:00 2012"),
    (32, "Mon Dec 31 23:59:45 2012", 15 * S, "Tue Jan 1 00:00:00 2013"),
    (35, "Mon Jul 9 14:45 2012", 15 * M + 50 * NS, "Mon Jul 9 15:00 2012"),
    (38, "Mon Jul 9 14:45:00 2012", 15 * MS, "Mon Jul 9 14:45:01 2012"),
    (41, "Mon Jul 9 14:45:00.005 2012", 15 * M, "Mon Jul 9 15:00 2012"),
    (44, "Mon Jul 9 14:45:00.005 2012", 15 * M + 50 * NS, "Mon Jul 9 15:00 2012"),
]

# ---- parser_test.go:18-41 TestRange: (line, expr, min, max, expected, err) ----
RANGE = [
    (18, "5", 0, 7, 1 << 5, ""),
    (19, "0", 0, 7, 1 << 0, ""),
    (20, "7", 0, 7, 1 << 7, ""),
    (22, "5-5", 0, 7, 1 << 5, ""),
    (23, "5-6", 0, 7, 1 << 5 | 1 << 6, ""),
    (24, "5-7", 0, 7, 1 << 5 | 1 << 6 | 1 << 7, ""),
    (26, "5-6/2", 0, 7, 1 << 5, ""),
    (27, "5-7/2", 0, 7, 1 << 5 | 1 << 7, ""),
    (28, "5-7/1", 0, 7, 1 << 5 | 1 << 6 | 1 << 7, ""),
    (30, "*", 1, 3, 1 << 1 | 1 << 2 | 1 << 3 | STAR, ""),
    (31, "*/2", 1, 3, 1 << 1 | 1 << 3 | STAR, ""),
    (33, "5--5", 0, 0, 0, "Too many hyphens"),
    (34, "jan-x", 0, 0, 0, "Failed to parse int from"),
    (35, "2-x", 1, 5, 0, "Failed to parse int from"),
    (36, "*/-12", 0, 0, 0, "Negative number"),
    (37, "*//2", 0, 0, 0, "Too many slashes"),
    (38, "1", 3, 5, 0, "below minimum"),
    (39, "6", 3, 5, 0, "above maximum"),
    (40, "5-3", 3, 5, 0, "beyond end of range"),
    (41, "*/0", 0, 0, 0, "should be a positive number"),
]

# ---- parser_test.go:64-67 TestField ----
FIELD = [
    (64, "5", 1, 7, 1 << 5),
    (65, "5,6", 1, 7, 1 << 5 | 1 << 6),
    (66, "5,6,7", 1, 7, 1 << 5 | 1 << 6 | 1 << 7),
    (67, "1,5-7/2,3", 1, 7, 1 << 1 | 1 << 5 | 1 << 7 | 1 << 3),
]

# ---- parser_test.go:83-87 TestAll: (line, min, max, expected-without-star) ----
ALL = [
    (83, 0, 59, 0xFFFFFFFFFFFFFFF),
    (84, 0, 23, 0xFFFFFF),
    (85, 1, 31, 0xFFFFFFFE),
    (86, 1, 12, 0x1FFE),
    (87, 0, 6, 0x7F),
]

# ---- parser_test.go:104-107 TestBits ----
BITS = [(104, 0, 0, 1, 0x1), (105, 1, 1, 1, 0x2), (106, 1, 5, 2, 0x2A), (107, 1, 4, 2, 0xA)]


def all_(lo, hi):
    return ((1 << (hi + 1)) - 1) & ~((1 << lo) - 1) | STAR


def spec(sec, mn, hr, dom, mon, dow):
    return {"kind": "spec", "second": sec, "minute": mn, "hour": hr,
            "dom": dom, "month": mon, "dow": dow}


SECS, MINS, HOURS, DOM, MONTHS, DOW = (0, 59), (0, 59), (0, 23), (1, 31), (1, 12), (0, 6)

# ---- parser_test.go:125-177 TestParse (default parser) ----
PARSE = [
    (126, "* 5 * * * *", spec(all_(*SECS), 1 << 5, all_(*HOURS), all_(*DOM), all_(*MONTHS), all_(*DOW)), ""),
    (137, "* 5 j * * *", None, "Failed to parse int from"),
    (141, "@every 5m", {"kind": "every", "delay_ns": 5 * M}, ""),
    (145, "@every Xm", None, "Failed to parse duration"),
    (149, "@yearly", spec(1, 1, 1, 1 << 1, 1 << 1, all_(*DOW)), ""),
    (160, "@annually", spec(1, 1, 1, 1 << 1, 1 << 1, all_(*DOW)), ""),
    (171, "@unrecognized", None, "Unrecognized descriptor"),
    (175, "* * * *", None, "Expected 5 to 6 fields"),
]

# ---- parser_test.go:200-215 TestStandardSpecSchedule (ParseStandard) ----
PARSE_STANDARD = [
    (201, "5 * * * *", spec(1, 1 << 5, all_(*HOURS), all_(*DOM), all_(*MONTHS), all_(*DOW)), ""),
    (205, "@every 5m", {"kind": "every", "delay_ns": 5 * M}, ""),
    (209, "5 j * * *", None, "Failed to parse int from"),
    (213, "* * * *", None, "Expected exactly 5 fields"),
]


def main():
    out = {"_source": "qlchan/cronsun node/cron/*_test.go (see gen_kats.py)",
           "zero_time": ZERO, "activation": [], "next": [], "errors": [],
           "next_tz": [], "constant_delay": [], "range": [], "field": [],
           "all": [], "bits": [], "parse": [], "parse_standard": []}
    for line, t, sp, exp in ACTIVATION:
        u, _, _ = parse_time(t)
        out["activation"].append({"ref": f"spec_test.go:{line}", "spec": sp,
                                  "time": u, "zone": "UTC", "expected": exp})
    for line, t, sp, exp in NEXT:
        u, _, off = parse_time(t)
        e, _, _ = parse_time(exp)
        zone = "America/New_York" if off is not None else "UTC"
        out["next"].append({"ref": f"spec_test.go:{line}", "spec": sp, "time": u,
                            "zone": zone, "expected": e})
    for line, sp in ERRORS:
        out["errors"].append({"ref": f"spec_test.go:{line}", "spec": sp})
    for line, t, sp, exp in NEXT_TZ:
        u, _, off = parse_time(t)
        e, _, _ = parse_time(exp)
        out["next_tz"].append({"ref": f"spec_test.go:{line}", "spec": sp, "time": u,
                               "zone": f"fixed:{off}", "expected": e})
    for line, t, d, exp in CONST_DELAY:
        u, ns, _ = parse_time(t)
        e, ens, _ = parse_time(exp)
        assert ens == 0
        out["constant_delay"].append({"ref": f"constantdelay_test.go:{line}", "time": u,
                                      "nsec": ns, "delay_ns": d, "expected": e})
    for line, expr, lo, hi, exp, err in RANGE:
        out["range"].append({"ref": f"parser_test.go:{line}", "expr": expr, "min": lo,
                             "max": hi, "expected": str(exp), "err": err})
    for line, expr, lo, hi, exp in FIELD:
        out["field"].append({"ref": f"parser_test.go:{line}", "expr": expr, "min": lo,
                             "max": hi, "expected": str(exp)})
    for line, lo, hi, exp in ALL:
        out["all"].append({"ref": f"parser_test.go:{line}", "min": lo, "max": hi,
                           "expected": str(exp | STAR)})
    for line, lo, hi, step, exp in BITS:
        out["bits"].append({"ref": f"parser_test.go:{line}", "min": lo, "max": hi,
                            "step": step, "expected": str(exp)})

    def enc(v):
        if v is None:
            return None
        return {k: (str(x) if isinstance(x, int) and k != "delay_ns" else x) for k, x in v.items()}

    for key, table in (("parse", PARSE), ("parse_standard", PARSE_STANDARD)):
        for line, expr, exp, err in table:
            out[key].append({"ref": f"parser_test.go:{line}", "expr": expr,
                             "expected": enc(exp), "err": err})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    n = sum(len(v) for k, v in out.items() if isinstance(v, list))
    print(f"wrote {path}: {n} rows")


if __name__ == "__main__":
    main()
