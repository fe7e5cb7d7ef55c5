"""test adaptor for the NaN watchdog: poisons the velocities after the first iteration"""


def initialize(constants):
    pass


def execute(fields, iteration, time, box):
    if iteration == 1:
        fields["vx"][0] = float("nan")


def finalize():
    pass
