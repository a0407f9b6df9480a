def jit(*a, **k):
    if a and callable(a[0]) and not k:
        return a[0]
    return lambda f: f
