"""Loopback ports for test servers and gangs.

An OS-assigned ephemeral port is free when it is picked but can be taken by
any socket that binds port 0 before the test's server binds it -- the gangs
under test open gloo / rendezvous sockets in exactly that window.  Ports here
come from below the kernel's ephemeral range and are never handed out twice
in one test process."""
import random
import socket

_TAKEN = set()


def free_port() -> int:
    try:
        lo = int(open("/proc/sys/net/ipv4/ip_local_port_range").read().split()[0])
    except (OSError, ValueError, IndexError):
        lo = 32768
    hi = max(20001, min(lo, 32768))
    for _ in range(1000):
        port = random.randrange(20000, hi)
        if port in _TAKEN:
            continue
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
        _TAKEN.add(port)
        return port
    with socket.socket() as s:  # range exhausted: fall back to the OS
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
