"""Share preparation oracle: ChaCha20 pinned by the
RFC 8439 test vectors, ChaCha8/12/20 by the published all-zero key/nonce block
(draft-strombergson-chacha-test-vectors, TC1), the C and numpy restatements
agree, and the shares satisfy EncodedBits::share's identity
(src/encoded_bits.rs:23-38).  12 rounds is the default: the reference's
thread_rng (rand 0.8.5) runs rand_chacha 0.3.1's ChaCha12."""
import numpy as np

from oracle import oracle_c as oc
from oracle import oracle_np as on

KEY = bytes(range(32))
# RFC 8439 §2.3.2 (block function): nonce 00:00:00:09:00:00:00:4a:00:00:00:00, counter 1,
# i.e. DJB counter64 = words 12-13 = 0x09000000_00000001, nonce64 = words 14-15 = 0x4a000000
RFC_BLOCK = bytes.fromhex(
    "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
    "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")
# RFC 8439 §2.4.2 (encryption): nonce 00:00:00:00:00:00:00:4a:00:00:00:00, initial counter 1
RFC_PLAIN = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for "
             b"the future, sunscreen would be it.")
RFC_CIPHER = bytes.fromhex(
    "6e2e359a2568f98041ba0728dd0d6981e97e7aec1d4360c20a27afccfd9fae0b"
    "f91b65c5524733ab8f593dabcd62b3571639d624e65152ab8f530c359f0861d8"
    "07ca0dbf500d6a6156a38e088a22b65e52bc514d16ccf806818ce91ab7793736"
    "5af90bbf74a35be6b40b8eedf2785e42874d")
# key 0^256, nonce 0^64, block 0 (draft-strombergson-chacha-test-vectors-00 TC1)
ZERO_BLOCK = {
    8: bytes.fromhex("3e00ef2f895f40d67f5bb8e81f09a5a12c840ec3ce9a7f3b181be188ef711a1e"
                     "984ce172b9216f419f445367456d5619314a42a3da86b001387bfdb80e0cfe42"),
    12: bytes.fromhex("9bf49a6a0755f953811fce125f2683d50429c3bb49e074147e0089a52eae155f"
                      "0564f879d27ae3c02ce82834acfa8c793a629f2ca0de6919610be82f411326be"),
    20: bytes.fromhex("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                      "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586"),
}


def test_chacha20_rfc8439_block():
    assert oc.chacha_block(KEY, 0x4A000000, 0x0900000000000001) == RFC_BLOCK
    assert on.chacha_blocks(KEY, 0x4A000000, [0x0900000000000001])[0].tobytes() == RFC_BLOCK


def test_chacha_zero_key_rounds():
    for rounds, want in ZERO_BLOCK.items():
        assert oc.chacha_block(bytes(32), 0, 0, rounds) == want, rounds
        assert on.chacha_blocks(bytes(32), 0, [0], rounds)[0].tobytes() == want, rounds


def test_chacha20_rfc8439_encryption():
    ks = oc.chacha_block(KEY, 0x4A000000, 1) + oc.chacha_block(KEY, 0x4A000000, 2)
    assert bytes(a ^ b for a, b in zip(RFC_PLAIN, ks)) == RFC_CIPHER


def test_chacha_c_vs_numpy():
    rng = np.random.default_rng(3)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    ctr = [0, 1, 2**32 - 1, 2**32, 2**63 + 5, 2**64 - 1]
    for rounds in (8, 12, 20):
        got = on.chacha_blocks(key, 0xDEADBEEF12345678, ctr, rounds)
        for i, c in enumerate(ctr):
            assert got[i].tobytes() == oc.chacha_block(key, 0xDEADBEEF12345678, c, rounds)


def test_prepare_c_vs_numpy_and_identity():
    t = oc.gen_templates(12, 0, 3)
    key = bytes(range(100, 132))
    for parties, rounds in ((1, 12), (2, 12), (3, 12), (3, 20), (2, 8)):
        s_c, m_c = oc.prepare_shares(t, key, nonce=7, parties=parties, index_base=1000, rounds=rounds)
        s_n, m_n = on.prepare_shares(t, key, nonce=7, parties=parties, index_base=1000, rounds=rounds)
        assert (s_c == s_n).all() and (m_c == m_n).all() and (m_c == t[:, 200:]).all()
        total = s_c.astype(np.uint64).sum(axis=0) % 65536
        enc = np.stack([oc.encode(x) for x in t])
        assert (total == enc).all()                       # sum of shares = encode (mod 2^16)
        if parties > 1:
            assert not (s_c[0] == enc).all()              # a random share reveals nothing directly
            assert (s_c[0][0] != s_c[0][1]).any()         # distinct keystream per template


def test_prepare_stream_independent_of_batching():
    """Template g's shares depend only on (key, nonce, g): preparing [0, 4) at once equals
    preparing each template alone at its index (what lets shards prepare independently)."""
    t = oc.gen_templates(13, 0, 4)
    key = bytes(32)
    whole, _ = oc.prepare_shares(t, key, parties=3, index_base=50)
    for i in range(4):
        one, _ = oc.prepare_shares(t[i:i + 1], key, parties=3, index_base=50 + i)
        assert (one[:, 0] == whole[:, i]).all()


def test_prepare_shares_look_uniform():
    t = oc.gen_templates(14, 0, 8)
    s, _ = oc.prepare_shares(t, bytes(range(32)), parties=3)
    x = s[:2].reshape(-1)
    # 204 800 u16 per share pair: mean ~ 32767.5, every byte value seen, no bias in the low bit
    assert abs(x.mean() - 32767.5) < 300
    assert np.unique(x & 0xFF).size == 256
    assert abs((x & 1).mean() - 0.5) < 0.01
