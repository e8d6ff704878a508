"""Enumerations and fixed constants of the order-book domain.

Restates ``gymnax_exchange/jaxob/jaxob_constants.py:1-91`` (values, not code):
message types, order-slot / trade-row field indices, cancel modes and the
interpretation of LOBSTER type-4 (execution) messages.  The integer values are
part of the drop-in contract (they appear in configs and in message arrays).
"""
from enum import IntEnum


class MaxInt(IntEnum):                     # jaxob_constants.py:3-5
    _64_Bit_Signed = 2_147_483_647         # (sic) the int32 maximum
    _32_Bit_Signed = 32_767


INITID = -2                                # jaxob_constants.py:8
NEGATIVE_RETURN_ID = -99
DUMMYID = -888888
EMPTY_SLOT = -1

ORDERBOOK_FEAT = 6                         # fields per order slot
TRADE_FEAT = 8                             # fields per trade row
MSG_FEAT = 8                               # fields per message row
NS_PER_SEC = 1e9

NTRADE_CAP = 100
NORDER_CAP = 100
STARTOFDAY = (34200, 0)
ENDOFDAY = (57600, 0)


class MessageType(IntEnum):                # jaxob_constants.py:28-35
    LIMIT = 1
    CANCEL = 2
    DELETE = 3
    MATCH = 4
    HIDDEN = 5
    AUCTION = 6
    HALT = 7


class OrderSideFeat(IntEnum):              # order slot row: [p, q, oid, tid, s, ns]
    P = 0
    Q = 1
    OID = 2
    TID = 3
    SEC = 4
    NSEC = 5


class TradesFeat(IntEnum):                 # trade row: [p, q, passOID, agrOID, s, ns, passTID, agrTID]
    P = 0
    Q = 1
    PASS_OID = 2
    AGRS_OID = 3
    SEC = 4
    NSEC = 5
    PASS_TID = 6
    AGRS_TID = 7


class LOBMSGFEAT(IntEnum):                 # message row: [type, side, q, p, oid, tid, s, ns]
    Type = 0
    Side = 1
    Quant = 2
    Price = 3
    OID = 4
    TID = 5
    TS = 6
    TNS = 7


class BidAskSide(IntEnum):
    BID = 1
    ASK = -1


class CancelMode(IntEnum):                 # jaxob_constants.py:64-68
    STRICT_BY_ID = 0
    INCLUDE_INITS = 1
    CANCEL_UNIFORM = 2
    CANCEL_UNIFORM_AND_LARGE = 3


class Type4Interpretation(IntEnum):        # jaxob_constants.py:70-74
    IOC = 0
    LIM = 1
    MKT = 2


class SimulatorMode(IntEnum):
    GENERAL_EXCHANGE = 0
    LOBSTER_INTERPRETER = 1


SEED = 42
