"""Literal pure-Python restatement of the witness-time big-integer functions of
circuits/lib/circuits/bigInt/bigIntFunc.circom, used to pin the C oracle's (and the GPU's)
quotient/remainder choice for BigMultModP.

TEST INFRASTRUCTURE ONLY (imported by tests/). Each function follows the cited reference
lines step by step (same loop bounds, same qhat corrections); circom field `var`s are Python
ints because every intermediate here stays far below p.
"""


def long_gt(n, k, a, b):  # bigIntFunc.circom:126-140
    for i in range(k - 1, -1, -1):
        if a[i] > b[i]:
            return 1
        if a[i] < b[i]:
            return 0
    return 0


def long_sub(n, k, a, b):  # bigIntFunc.circom:142-167
    diff = [0] * 200
    borrow = [0] * 200
    for i in range(k):
        if i == 0:
            if a[i] >= b[i]:
                diff[i] = a[i] - b[i]
                borrow[i] = 0
            else:
                diff[i] = a[i] - b[i] + (1 << n)
                borrow[i] = 1
        else:
            if a[i] >= b[i] + borrow[i - 1]:
                diff[i] = a[i] - b[i] - borrow[i - 1]
                borrow[i] = 0
            else:
                diff[i] = (1 << n) + a[i] - b[i] - borrow[i - 1]
                borrow[i] = 1
    return diff


def long_scalar_mult(n, k, a, b):  # bigIntFunc.circom:169-181
    out = [0] * 200
    for i in range(k):
        temp = out[i] + a * b[i]
        out[i] = temp % (1 << n)
        out[i + 1] = out[i + 1] + temp // (1 << n)
    return out


def short_div_norm(n, k, a, b):  # bigIntFunc.circom:290-312
    qhat = (a[k] * (1 << n) + a[k - 1]) // b[k - 1]
    if qhat > (1 << n) - 1:
        qhat = (1 << n) - 1
    mult = long_scalar_mult(n, k, qhat, b)
    if long_gt(n, k + 1, mult, a) == 1:
        mult = long_sub(n, k + 1, mult, b)
        if long_gt(n, k + 1, mult, a) == 1:
            return qhat - 2
        return qhat - 1
    return qhat


def short_div(n, k, a, b):  # bigIntFunc.circom:314-333
    scale = (1 << n) // (1 + b[k - 1])
    norm_a = long_scalar_mult(n, k + 1, scale, a)
    norm_b = long_scalar_mult(n, k, scale, b)
    if norm_b[k] != 0:
        return short_div_norm(n, k + 1, norm_a, norm_b)
    return short_div_norm(n, k, norm_a, norm_b)


def long_div(n, k, m, a, b):  # bigIntFunc.circom:190-232
    out = [[0] * 200 for _ in range(2)]
    remainder = [0] * 200
    for i in range(m + k):
        remainder[i] = a[i]
    dividend = [0] * 200
    for i in range(m, -1, -1):
        if i == m:
            dividend[k] = 0
            for j in range(k - 1, -1, -1):
                dividend[j] = remainder[j + m]
        else:
            for j in range(k, -1, -1):
                dividend[j] = remainder[j + i]
        out[0][i] = short_div(n, k, dividend, b)
        mult_shift = long_scalar_mult(n, k, out[0][i], b)
        subtrahend = [0] * 200
        for j in range(k + 1):
            if i + j < m + k:
                subtrahend[i + j] = mult_shift[j]
        remainder = long_sub(n, m + k, remainder, subtrahend)
    for i in range(k):
        out[1][i] = remainder[i]
    out[1][k] = 0
    return out


def reduce_overflow(n, k, m, N):  # bigIntFunc.circom:570-588
    M = [0] * 200
    overflow = 0
    for i in range(k):
        if i == 0:
            M[i] = N[i] % (2 ** n)
            overflow = N[i] // (2 ** n)
        else:
            M[i] = (N[i] + overflow) % (2 ** n)
            overflow = (N[i] + overflow) // (2 ** n)
    for i in range(k, m):
        M[i] = overflow % (2 ** n)
        overflow = overflow // (2 ** n)
    return M


def big_mult_mod_p_divmod(x_limbs, y_limbs, mod_limbs, n=64):
    """div, mod exactly as BigMultModP (bigInt.circom:224-238) obtains them."""
    K = len(mod_limbs)
    G, L = len(x_limbs), len(y_limbs)
    base = G + L
    prod = [0] * (base - 1)
    for i in range(G):
        for j in range(L):
            prod[i + j] += x_limbs[i] * y_limbs[j]
    reduced = reduce_overflow(n, base - 1, base, prod)
    DIV = base - K + 1
    res = long_div(n, K, DIV - 1, reduced, mod_limbs)
    return res[0][:DIV], res[1][:K]
