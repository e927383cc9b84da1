"""``posggym.utils.history`` stand-in for the reference harness (TEST INFRASTRUCTURE).

posggym is not installed; ``INTMCP`` and ``MCTS`` with
``state_belief_only=False`` use its ``AgentHistory`` / ``JointHistory``.  Only
the operations the reference calls are restated:
``get_init_history``, ``extend``, ``get_agent_history``, ``get_last_step``,
iteration over (action, obs) steps, ``.history``, hashing and equality."""


class AgentHistory:
    __slots__ = ("history",)

    def __init__(self, history):
        self.history = tuple(history)

    @classmethod
    def get_init_history(cls, obs=None):
        return cls(()) if obs is None else cls(((None, obs),))

    def extend(self, action, obs):
        return AgentHistory(self.history + ((action, obs),))

    def get_last_step(self):
        return self.history[-1]

    def __iter__(self):
        return iter(self.history)

    def __len__(self):
        return len(self.history)

    def __hash__(self):
        return hash(self.history)

    def __eq__(self, other):
        return isinstance(other, AgentHistory) and self.history == other.history

    def __repr__(self):
        return f"AgentHistory({self.history})"


class JointHistory:
    __slots__ = ("agent_ids", "agent_histories")

    def __init__(self, agent_ids, agent_histories):
        self.agent_ids = tuple(agent_ids)
        self.agent_histories = tuple(agent_histories)

    @classmethod
    def get_init_history(cls, agent_ids, initial_joint_obs=None):
        if initial_joint_obs is None:
            return cls(agent_ids, [AgentHistory.get_init_history() for _ in agent_ids])
        return cls(agent_ids, [AgentHistory.get_init_history(initial_joint_obs[i])
                               for i in agent_ids])

    def extend(self, joint_action, joint_obs):
        return JointHistory(self.agent_ids, [h.extend(joint_action[i], joint_obs[i])
                                             for i, h in zip(self.agent_ids, self.agent_histories)])

    def get_agent_history(self, agent_id):
        return self.agent_histories[self.agent_ids.index(agent_id)]

    def __hash__(self):
        return hash(self.agent_histories)

    def __eq__(self, other):
        return isinstance(other, JointHistory) and self.agent_histories == other.agent_histories
