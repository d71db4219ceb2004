"""Robot / Perception surfaces of rfarl's WAM-V model (rfarl/rfarl/envs/marinenav/vehicles/wamv.py).

These objects hold the per-robot state and parameters exactly as the reference's Robot does
(same attribute names, same defaults, same per-robot numpy RandomState for perception noise),
so Trainer code and eval tooling that read or write them keep working. The physics that the
reference runs in Robot.update_state / compute_motion / perception_output (wamv.py:204-529)
is executed by the gfx950 env-step kernel through MarineNavEnv3.step; those methods are not
provided here.
"""
import numpy as np


class Perception:
    """wamv.py:5-40: sector 'LiDAR' parameters and the per-robot noise generator."""

    def __init__(self, seed: int = 0):
        self.seed = seed
        self.rd = np.random.RandomState(seed)
        self.range = 20.0
        self.angle = 2 * np.pi
        self.max_obj_num = 5
        self.observation = dict(self=[], objects=[])
        self.observed_obs = []
        self.observed_objs = []
        self.pos_std = 0.05
        self.vel_std = 0.05
        self.r_kappa = 1.0
        self.r_mean_ratio = 0.8

    def draw_candidate_noise(self):
        """The five draws one detection candidate consumes, in the reference's order:
        pos_observation (2 normals), vel_observation (2 normals), r_observation (von Mises)
        (wamv.py:27-40, called at :466-468 and :493-495)."""
        rd = self.rd
        return (rd.normal(0, self.pos_std), rd.normal(0, self.pos_std), rd.normal(0, self.vel_std),
                rd.normal(0, self.vel_std), rd.vonmises(0, self.r_kappa))


class Robot:
    """wamv.py:43-145 state, parameters and bookkeeping of one WAM-V."""

    def __init__(self, seed: int = 0):
        self.dt = 0.05
        self.N = 10
        self.perception = Perception(seed)
        self.length = 5.0
        self.width = 2.5
        self.detect_r = 0.5 * np.sqrt(self.length ** 2 + self.width ** 2)
        self.r = self.detect_r
        self.head_on_zone_x_dim = 17.0
        self.head_on_zone_y_dim = 9.0
        self.left_crossing_zone_x_dim = np.array([-9.0, 12.0])
        self.left_crossing_zone_y_dim_front = np.array([-17.0, -7.0])
        self.safe_dis = 10.0
        self.goal_dis = 2.0
        self.goal_angluar_speed = np.pi / 12
        self.max_angular_speed = np.pi / 3
        self.power_coefficient = 1.0
        self.min_thrust = -500.0
        self.max_thrust = 1000.0
        self.left_thrust_change = np.array([0.0, -500.0, -1000.0, 500.0, 1000.0])
        self.right_thrust_change = np.array([0.0, -500.0, -1000.0, 500.0, 1000.0])
        self.compute_actions()
        self.x = None
        self.y = None
        self.theta = None
        self.velocity_r = None
        self.velocity = None
        self.left_pos = None
        self.right_pos = None
        self.left_thrust = None
        self.right_thrust = None
        self.m = 400
        self.Izz = 450
        self.xDotU = 20
        self.yDotV = 0
        self.yDotR = 0
        self.nDotR = -980
        self.nDotV = 0
        self.xU = -100
        self.xUU = -150
        self.yV = -100
        self.yVV = -150
        self.yR = 0
        self.yRV = 0
        self.yVR = 0
        self.yRR = 0
        self.nR = -980
        self.nRR = -950
        self.nV = 0
        self.nVV = 0
        self.nRV = 0
        self.nVR = 0
        self.compute_constant_matrices()
        self.start = None
        self.goal = None
        self.collision = False
        self.reach_goal = False
        self.deactivated = False
        self.apply_COLREGs = False
        self.phi = 0.0
        self.init_theta = 0.0
        self.init_velocity_r = np.array([0.0, 0.0, 0.0])
        self.init_left_pos = 0.0
        self.init_right_pos = 0.0
        self.init_left_thrust = 0.0
        self.init_right_thrust = 0.0
        self.observation_history = []
        self.action_history = []
        self.trajectory = []

    def compute_actions(self):  # wamv.py:146-147
        self.actions = [(l, r) for l in self.left_thrust_change for r in self.right_thrust_change]

    def compute_actions_dimension(self):
        return len(self.actions)

    def compute_constant_matrices(self):  # wamv.py:152-159
        self.M_RB = np.array([[self.m, 0.0, 0.0], [0.0, self.m, 0.0], [0.0, 0.0, self.Izz]])
        self.M_A = -1.0 * np.array([[self.xDotU, 0.0, 0.0], [0.0, self.yDotV, self.yDotR],
                                    [0.0, self.nDotV, self.nDotR]])
        self.D = -1.0 * np.array([[self.xU, 0.0, 0.0], [0.0, self.yV, self.yR], [0.0, self.nV, self.nR]])

    def compute_step_energy_cost(self):  # wamv.py:161-165
        l = self.power_coefficient * np.abs(self.left_thrust) * self.dt * self.N
        r = self.power_coefficient * np.abs(self.right_thrust) * self.dt * self.N
        return l + r

    def dist_to_goal(self):
        return np.linalg.norm(self.goal - np.array([self.x, self.y]))

    def check_over_spin(self):
        return np.abs(self.velocity[2]) > self.max_angular_speed

    def reset_state(self, current_velocity=np.zeros(3)):  # wamv.py:177-193
        self.observation_history.clear()
        self.action_history.clear()
        self.trajectory.clear()
        self.x = self.start[0]
        self.y = self.start[1]
        self.theta = self.init_theta
        self.velocity_r = self.init_velocity_r
        self.velocity = self.velocity_r + current_velocity
        self.left_pos = self.init_left_pos
        self.right_pos = self.init_right_pos
        self.left_thrust = self.init_left_thrust
        self.right_thrust = self.init_right_thrust
        self.trajectory.append(self.trajectory_row())

    def trajectory_row(self):  # wamv.py:191-193, env.py:267-269
        return [self.x, self.y, self.theta, self.velocity_r[0], self.velocity_r[1], self.velocity_r[2],
                self.velocity[0], self.velocity[1], self.velocity[2], self.left_pos, self.right_pos,
                self.left_thrust, self.right_thrust]

    def physics_signature(self):
        """Parameters the env-step kernel takes once per batch (AsvParams)."""
        per = self.perception
        return (self.dt, self.N, self.length, self.width, self.r, self.goal_dis, self.min_thrust, self.max_thrust,
                self.m, self.Izz, self.xDotU, self.yDotV, self.yDotR, self.nDotR, self.nDotV, self.xU, self.xUU,
                self.yV, self.yVV, self.yR, self.yRV, self.yVR, self.yRR, self.nR, self.nRR, self.nV, self.nVV,
                self.nRV, self.nVR, tuple(self.left_thrust_change), tuple(self.right_thrust_change), per.range,
                per.angle, per.max_obj_num, per.pos_std, per.vel_std, per.r_kappa, per.r_mean_ratio)
