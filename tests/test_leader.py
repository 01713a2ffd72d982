"""Lease-based leader election (ncc/leader.py): a capability the reference lacks (single replica only,
.helm/templates/deployment.yaml:15-19; SURVEY.md §5.3 "HA: none")."""
import asyncio

from ncc.api import resources as R
from ncc.fakeapi.storage import ClusterState
from ncc.kube import errors as E
from ncc.leader import LeaderElector
from ncc.testing.fake_client import FakeClient

NS = "nexus"


class Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def pair(clock):
    st = ClusterState("c")
    mk = lambda ident: LeaderElector(FakeClient(st, simple=False), NS, "ncc", ident, lease_duration=15,  # noqa: E731
                                     renew_deadline=10, retry_period=2, clock=clock)
    return st, mk("a"), mk("b")


async def test_only_one_candidate_leads_and_takeover_after_expiry():
    clock = Clock()
    st, a, b = pair(clock)
    assert await a.try_acquire_or_renew() and a.leading
    assert not await b.try_acquire_or_renew()
    lease = st.get(R.LEASES, NS, "ncc")
    assert lease["spec"]["holderIdentity"] == "a" and lease["spec"]["leaseDurationSeconds"] == 15
    # a renews: b keeps seeing fresh renewTimes, so the lease never looks expired to b
    clock.t = 10
    assert await a.try_acquire_or_renew()
    clock.t = 20
    assert not await b.try_acquire_or_renew()
    # a dies (stops renewing): b takes over once lease_duration passed since b last saw a change
    clock.t = 36
    assert await b.try_acquire_or_renew() and b.leading
    lease = st.get(R.LEASES, NS, "ncc")
    assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] == 1
    # a comes back: it must not steal the lease, and learns it no longer leads
    assert not await a.try_acquire_or_renew() and not a.leading


async def test_release_hands_over_immediately():
    clock = Clock()
    st, a, b = pair(clock)
    assert await a.try_acquire_or_renew()
    assert not await b.try_acquire_or_renew()
    assert await a.release() and not a.leading
    assert st.get(R.LEASES, NS, "ncc")["spec"]["holderIdentity"] == ""
    assert await b.try_acquire_or_renew()


async def test_conflicting_writes_have_one_winner():
    clock = Clock()
    st, a, b = pair(clock)
    # both read "no lease"; both create; exactly one create succeeds
    wins = await asyncio.gather(a.try_acquire_or_renew(), b.try_acquire_or_renew())
    assert sorted(wins) == [False, True]


async def test_hold_reports_loss_after_renew_deadline():
    clock = Clock()
    st = ClusterState("c")
    client = FakeClient(st, simple=False)
    a = LeaderElector(client, NS, "ncc", "a", lease_duration=0.3, renew_deadline=0.2, retry_period=0.05)
    assert await a.acquire()
    client.prepend_reactor("*", "leases", lambda act: (True, None, E.ServiceUnavailable("apiserver down")))
    lost = asyncio.Event()
    await asyncio.wait_for(a.hold(None, on_lost=lost.set), 2.0)
    assert lost.is_set() and not a.leading


async def test_hold_bounds_a_hanging_renew_by_the_renew_deadline():
    """a renew that hangs (slow apiserver, Retry-After back-off) must not outlive renew_deadline;
    otherwise a standby could take the expired Lease while this replica still believes it leads."""
    st = ClusterState("c")
    client = FakeClient(st, simple=False)
    a = LeaderElector(client, NS, "ncc", "a", lease_duration=0.5, renew_deadline=0.3, retry_period=0.05)
    assert await a.acquire()
    orig_get = client.get

    async def hanging_get(*args, **kw):
        await asyncio.sleep(30)
        return await orig_get(*args, **kw)
    client.get = hanging_get
    lost = asyncio.Event()
    loop = asyncio.get_running_loop()
    t0 = loop.time()
    await asyncio.wait_for(a.hold(None, on_lost=lost.set), 2.0)
    assert lost.is_set() and not a.leading
    assert loop.time() - t0 < 0.5  # gave up inside the lease duration, not after the hung request
