class _Flags(object):
    def __call__(self, argv):
        return argv


FLAGS = _Flags()
