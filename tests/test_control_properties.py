"""Property-based tests of the control plane's pure logic (hypothesis instead of the
reference's example-only unit tests): secret encryption, password hashing, cron matching, inventory host
patterns and YAML round trip, free-form module argument parsing, and the zone IP pool as a state machine."""
import datetime as dt
import ipaddress

import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402
from hypothesis.stateful import RuleBasedStateMachine, invariant, precondition, rule  # noqa: E402

from kubeoperator_amd.control.engine.inventory import Inventory  # noqa: E402
from kubeoperator_amd.control.engine.runner import _parse_free_form, _split_top_level  # noqa: E402
from kubeoperator_amd.control.runtime.scheduler import cron_match  # noqa: E402
from kubeoperator_amd.control.store import crypto  # noqa: E402

PROPS = settings(max_examples=60, deadline=None, derandomize=True)


@PROPS
@given(plain=st.text(min_size=1, max_size=200), secret=st.text(min_size=1, max_size=40))
def test_encrypt_roundtrip_and_tamper(plain, secret):
    tok = crypto.encrypt(plain, secret)
    if plain.startswith(crypto.PREFIX):
        assert tok == plain
        return
    assert tok.startswith(crypto.PREFIX) and tok != crypto.encrypt(plain, secret)  # fresh nonce per call
    assert crypto.decrypt(tok, secret) == plain
    with pytest.raises(ValueError):
        crypto.decrypt(tok, secret + "x")
    import base64
    raw = bytearray(base64.urlsafe_b64decode(tok[len(crypto.PREFIX):]))
    raw[-1] ^= 1
    with pytest.raises(ValueError):
        crypto.decrypt(crypto.PREFIX + base64.urlsafe_b64encode(bytes(raw)).decode(), secret)


@settings(max_examples=15, deadline=None, derandomize=True)
@given(pw=st.text(max_size=40), other=st.text(max_size=40))
def test_password_hash_verifies_only_itself(pw, other):
    enc = crypto.hash_password(pw, iterations=1000)
    assert crypto.verify_password(pw, enc)
    assert crypto.verify_password(other, enc) == (other == pw)
    assert not crypto.verify_password(pw, "md5$1$x$y")


_times = st.datetimes(min_value=dt.datetime(2020, 1, 1), max_value=dt.datetime(2030, 12, 31))


@PROPS
@given(t=_times, step=st.integers(1, 30), lo=st.integers(0, 23), span=st.integers(0, 23))
def test_cron_fields(t, step, lo, span):
    hi = min(23, lo + span)
    assert cron_match("* * * * *", t)
    assert cron_match(f"*/{step} * * * *", t) == (t.minute % step == 0)
    assert cron_match(f"0 {lo}-{hi} * * *", t) == (t.minute == 0 and lo <= t.hour <= hi)
    assert cron_match(f"{t.minute},{(t.minute + 7) % 60} {t.hour} {t.day} {t.month} *", t)
    dow = (t.weekday() + 1) % 7  # cron: 0 = Sunday
    assert cron_match(f"* * * * {dow}", t) and not cron_match(f"* * * * {(dow + 1) % 7}", t)


# ----------------------------------------------------------------------------------------------- inventory
@st.composite
def inventories(draw):
    hosts = [f"h{i}" for i in range(draw(st.integers(1, 8)))]
    groups = [f"g{i}" for i in range(draw(st.integers(1, 5)))]
    inv = Inventory()
    members = {}
    for h in hosts:
        gs = draw(st.lists(st.sampled_from(groups), unique=True, max_size=3))
        inv.add_host(h, {"ansible_host": f"10.0.0.{len(members) + 1}", "idx": len(members)}, groups=gs)
        members[h] = set(gs)
    # children only point to later groups: a DAG
    children = {g: draw(st.lists(st.sampled_from(groups[i + 1:]), unique=True, max_size=2)) if i + 1 < len(groups)
                else [] for i, g in enumerate(groups)}
    for g in groups:
        inv.add_group(g, {"gv": g}, children=children[g])
    return inv, hosts, groups, members, children


def _expected(g, members, children):
    out = {h for h, gs in members.items() if g in gs}
    for c in children[g]:
        out |= _expected(c, members, children)
    return out


@PROPS
@given(data=inventories())
def test_inventory_groups_patterns_roundtrip(data):
    inv, hosts, groups, members, children = data
    for g in groups:
        assert set(inv.group_hosts(g)) == _expected(g, members, children)
    assert inv.match("all") == hosts
    a, b = groups[0], groups[-1]
    ea, eb = _expected(a, members, children), _expected(b, members, children)
    assert set(inv.match(f"{a}:{b}")) == ea | eb
    assert set(inv.match(f"{a}:&{b}")) == ea & eb
    assert set(inv.match(f"{a}:!{b}")) == ea - eb
    order = inv.match(f"{a}:{b}")
    assert order == sorted(order, key=hosts.index)
    if inv.group_hosts(a):
        assert inv.match(f"{a}[0]") == inv.group_hosts(a)[:1]
    back = Inventory.from_dict(inv.to_dict())
    for g in groups:
        assert set(back.group_hosts(g)) == set(inv.group_hosts(g))
    for h in hosts:
        assert back.host_vars(h)["idx"] == inv.host_vars(h)["idx"]


# ------------------------------------------------------------------------------------ free-form arguments
_key = st.from_regex(r"[a-z_][a-z0-9_]{0,8}", fullmatch=True)
_plain = st.from_regex(r"[A-Za-z0-9_./:-]{1,12}", fullmatch=True)
_quoted = st.builds(lambda w: f'"{w}"', st.from_regex(r"[A-Za-z0-9 ,./-]{1,12}", fullmatch=True))
_jinja = st.builds(lambda v: "{{ " + v + " }}", st.sampled_from(["inventory_hostname", "x | default('a b')",
                                                                     "groups['kube-master'][0]"]))


@PROPS
@given(pairs=st.dictionaries(_key, st.one_of(_plain, _quoted, _jinja), min_size=1, max_size=5))
def test_free_form_key_values(pairs):
    s = " ".join(f"{k}={v}" for k, v in pairs.items())
    assert len(_split_top_level(s)) == len(pairs)
    got = _parse_free_form("copy", s)
    want = {k: (v[1:-1] if v.startswith('"') else v) for k, v in pairs.items()}
    assert got == want


@PROPS
@given(cmd=st.from_regex(r"[a-z]{1,6}( [a-z0-9-]{1,6}){0,4}", fullmatch=True))
def test_free_form_command_keeps_raw(cmd):
    assert _parse_free_form("shell", cmd + " chdir=/tmp") == {"chdir": "/tmp", "_raw_params": cmd}
    assert _parse_free_form("debug", cmd) == {"msg": cmd}


# ----------------------------------------------------------------------------------- IP pool state machine
def test_ip_pool_state_machine(control):
    from kubeoperator_amd.control.domain import cloud
    from kubeoperator_amd.control.store import models as M
    from kubeoperator_amd.control.store.db import session_scope

    with session_scope() as s:
        r = M.Region(name="r-prop", vars={"provider": "fake"})
        s.add(r)
        s.flush()
        z = M.Zone(name="z-prop", region_id=r.id, vars={"ip_start": "10.9.0.250", "ip_end": "10.9.1.4"})
        s.add(z)
        s.flush()
        zid = z.id
    pool = [str(ipaddress.ip_address(int(ipaddress.ip_address("10.9.0.250")) + i)) for i in range(11)]

    class IpPool(RuleBasedStateMachine):
        def __init__(self):
            super().__init__()
            self.held: list[str] = []
            with session_scope() as s:
                s.get(M.Zone, zid).ip_used = []

        @precondition(lambda self: len(self.held) < len(pool))
        @rule()
        def allocate(self):
            ip = cloud.allocate_ip(zid)
            assert ip in pool and ip not in self.held
            self.held.append(ip)

        @precondition(lambda self: len(self.held) == len(pool))
        @rule()
        def exhausted(self):
            with pytest.raises(RuntimeError):
                cloud.allocate_ip(zid)

        @precondition(lambda self: self.held)
        @rule(i=st.integers(0, 100))
        def recover(self, i):
            ip = self.held.pop(i % len(self.held))
            cloud.recover_ip(zid, ip)

        @invariant()
        def accounted(self):
            with session_scope() as s:
                z = s.get(M.Zone, zid)
                free = cloud.ip_pool(z, "fake")
                assert sorted(z.ip_used or []) == sorted(self.held)
            assert set(free) | set(self.held) == set(pool) and not set(free) & set(self.held)

    IpPool.TestCase.settings = settings(max_examples=25, stateful_step_count=30, deadline=None, derandomize=True,
                                        suppress_health_check=list(HealthCheck))
    IpPool.TestCase().runTest()
