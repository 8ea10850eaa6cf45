"""A rendezvous port for the multi-process tests, drawn below Linux's
ephemeral range (32768-60999): a port taken from bind(0) and released again
can be handed to one of the many outgoing connections the previous test's
ranks (gloo / RCCL) open before torchrun's store binds it -- rank 0 then
exits 1 and the others are killed (seen once in a full GPU suite, r05)."""
import random
import socket


def free_port():
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
        except OSError:
            continue
        finally:
            s.close()
        return p
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
