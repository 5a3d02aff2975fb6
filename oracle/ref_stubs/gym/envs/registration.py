def register(**kwargs):
    return None
