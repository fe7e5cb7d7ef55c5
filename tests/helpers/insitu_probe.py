"""test adaptor for --insitu: records what the driver passes"""
CALLS = []


def initialize(constants):
    CALLS.append(("init", sorted(constants)[:3]))


def execute(fields, iteration, time, box):
    CALLS.append(("exec", iteration, int(fields["x"].numel()), "rho" in fields or "temp" in fields))


def finalize():
    CALLS.append(("fin",))
