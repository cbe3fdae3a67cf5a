"""Exception types of the reference's hot-path boundary (src/exceptions/*.py)."""


class HiddenStateNotInitialized(Exception):
    def __init__(self):
        super().__init__("Please run init_hidden() to initialize the hidden state before running forward pass.)")


class MultiAgentControllerNotInitialized(Exception):
    def __init__(self):
        super().__init__("Multi-Agent Controller not initialized."
                         "Please run initialize() with it`s corresponding arguments to prepare the runner.")


class NoLearnersProvided(Exception):
    def __init__(self):
        super().__init__("The provided list of learners is empty. Make sure to register learners before calling a save.")
