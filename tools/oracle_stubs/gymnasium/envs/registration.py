def register(id, entry_point, **kw):
    import gymnasium
    gymnasium._REGISTRY[id] = entry_point
