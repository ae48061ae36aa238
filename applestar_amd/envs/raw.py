"""Plain-Python mirror of the subset of the SC2 API protobuf tree the agent reads.

The featurizer (:mod:`applestar_amd.agent.features`) only uses attribute access, so it accepts either
real ``s2clientprotocol`` messages (from :class:`~applestar_amd.envs.sc2_env.SC2Env`) or these
structures (from :class:`~applestar_amd.envs.fake_env.FakeSC2Env`).  Field names follow
``raw_pb2`` / ``sc2api_pb2`` / ``common_pb2`` / ``score_pb2`` so the two are interchangeable.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

# sc2api_pb2 enums used by the agent
RACE = {'random': 4, 'zerg': 2, 'terran': 1, 'protoss': 3}
RACE_NAME = {v: k for k, v in RACE.items()}
PLAYER_TYPE_PARTICIPANT, PLAYER_TYPE_COMPUTER, PLAYER_TYPE_OBSERVER = 1, 2, 3
RESULT_VICTORY, RESULT_DEFEAT, RESULT_TIE, RESULT_UNDECIDED = 1, 2, 3, 4


@dataclass
class Point:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0


@dataclass
class Size2D:
    x: int = 0
    y: int = 0


@dataclass
class ImageData:
    bits_per_pixel: int = 8
    size: Size2D = field(default_factory=Size2D)
    data: bytes = b''


@dataclass
class UnitOrder:
    ability_id: int = 0
    progress: float = 0.0


@dataclass
class PassengerUnit:
    tag: int = 0
    health: float = 0.0
    health_max: float = 0.0
    shield: float = 0.0
    shield_max: float = 0.0
    energy: float = 0.0
    energy_max: float = 0.0
    unit_type: int = 0


@dataclass
class Unit:
    display_type: int = 1
    alliance: int = 1
    tag: int = 0
    unit_type: int = 0
    owner: int = 1
    pos: Point = field(default_factory=Point)
    facing: float = 0.0
    radius: float = 0.5
    build_progress: float = 1.0
    cloak: int = 3
    is_blip: bool = False
    is_powered: bool = False
    is_active: bool = False
    attack_upgrade_level: int = 0
    armor_upgrade_level: int = 0
    shield_upgrade_level: int = 0
    health: float = 0.0
    health_max: float = 0.0
    shield: float = 0.0
    shield_max: float = 0.0
    energy: float = 0.0
    energy_max: float = 0.0
    mineral_contents: int = 0
    vespene_contents: int = 0
    is_flying: bool = False
    is_burrowed: bool = False
    is_hallucination: bool = False
    orders: List[UnitOrder] = field(default_factory=list)
    add_on_tag: int = 0
    passengers: List[PassengerUnit] = field(default_factory=list)
    cargo_space_taken: int = 0
    cargo_space_max: int = 0
    assigned_harvesters: int = 0
    ideal_harvesters: int = 0
    weapon_cooldown: float = 0.0
    buff_ids: List[int] = field(default_factory=list)


@dataclass
class Effect:
    effect_id: int = 0
    pos: List[Point] = field(default_factory=list)
    alliance: int = 1
    owner: int = 1
    radius: float = 1.0


@dataclass
class PlayerRaw:
    upgrade_ids: List[int] = field(default_factory=list)


@dataclass
class ObservationRaw:
    player: PlayerRaw = field(default_factory=PlayerRaw)
    units: List[Unit] = field(default_factory=list)
    effects: List[Effect] = field(default_factory=list)


@dataclass
class PlayerCommon:
    player_id: int = 1
    minerals: int = 50
    vespene: int = 0
    food_cap: int = 14
    food_used: int = 12
    food_army: int = 0
    food_workers: int = 12
    idle_worker_count: int = 0
    army_count: int = 0
    warp_gate_count: int = 0
    larva_count: int = 3


@dataclass
class CategoryScoreDetails:
    none: float = 0.0
    army: float = 0.0
    economy: float = 0.0
    technology: float = 0.0
    upgrade: float = 0.0


@dataclass
class ScoreDetails:
    killed_minerals: CategoryScoreDetails = field(default_factory=CategoryScoreDetails)
    killed_vespene: CategoryScoreDetails = field(default_factory=CategoryScoreDetails)


@dataclass
class Score:
    score_details: ScoreDetails = field(default_factory=ScoreDetails)


@dataclass
class MinimapRenders:
    height_map: ImageData = field(default_factory=ImageData)
    visibility_map: ImageData = field(default_factory=ImageData)
    creep: ImageData = field(default_factory=ImageData)
    player_relative: ImageData = field(default_factory=ImageData)
    alerts: ImageData = field(default_factory=ImageData)
    pathable: ImageData = field(default_factory=ImageData)
    buildable: ImageData = field(default_factory=ImageData)


@dataclass
class FeatureLayerData:
    minimap_renders: MinimapRenders = field(default_factory=MinimapRenders)


@dataclass
class Observation:
    game_loop: int = 0
    player_common: PlayerCommon = field(default_factory=PlayerCommon)
    raw_data: ObservationRaw = field(default_factory=ObservationRaw)
    feature_layer_data: FeatureLayerData = field(default_factory=FeatureLayerData)
    score: Score = field(default_factory=Score)


@dataclass
class ActionError:
    unit_tag: int = 0
    ability_id: int = 0
    result: int = 1


@dataclass
class PlayerResult:
    player_id: int = 1
    result: int = RESULT_UNDECIDED


@dataclass
class ResponseObservation:
    observation: Observation = field(default_factory=Observation)
    action_errors: List[ActionError] = field(default_factory=list)
    player_result: List[PlayerResult] = field(default_factory=list)


@dataclass
class PlayerInfo:
    player_id: int = 1
    type: int = PLAYER_TYPE_PARTICIPANT
    race_requested: int = RACE['zerg']
    race_actual: int = RACE['zerg']


@dataclass
class StartRaw:
    map_size: Size2D = field(default_factory=Size2D)
    start_locations: List[Point] = field(default_factory=list)


@dataclass
class GameInfo:
    map_name: str = ''
    player_info: List[PlayerInfo] = field(default_factory=list)
    start_raw: StartRaw = field(default_factory=StartRaw)


@dataclass
class RawUnitCommand:
    """Translated agent action (``raw_pb2.ActionRawUnitCommand``)."""
    ability_id: int = 0
    unit_tags: List[int] = field(default_factory=list)
    queue_command: bool = False
    target_unit_tag: int = 0
    target_world_space_pos: Point = None
